set -o pipefail
for v in ${LP_SIZES:-64 61 63 57}; do
  echo "== DLR_LONG_PIECE=$v"
  DLR_LONG_PIECE=$v bash tools/prof_c3.sh | grep -E "long_phase|long_combine" || exit 1
done
