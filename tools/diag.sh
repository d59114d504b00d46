#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for s in auto 16 32 64; do
  if [ $s = auto ]; then unset DLR_MARGIN_SEG; else export DLR_MARGIN_SEG=$s; fi
  timeout -k 5 120 python -u tools/diag_ragged.py 257 2>&1 | tail -4 || exit 1
done
