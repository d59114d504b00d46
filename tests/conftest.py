"""Shared test setup.

Markers: `gpu` = needs a real MI355X (parity tests through the C-ABI);
everything else runs on CPU in the build container.  Native libraries are
built in-tree on first use (make is incremental and takes seconds).
"""
from __future__ import annotations

import os
import subprocess
import sys

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, os.path.join(ROOT, "dist-lr_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD MI355X GPU (runs on the GPU box)")
    config.addinivalue_line("markers", "full: full-size case (minutes); runs only with DLR_FULL=1 -- the final "
                                       "tree's run, whose log is committed under profiles/")


def pytest_collection_modifyitems(config, items):
    if os.environ.get("DLR_FULL") == "1":
        return
    skip = pytest.mark.skip(reason="full-size case: set DLR_FULL=1")
    for it in items:
        if "full" in it.keywords:
            it.add_marker(skip)


def _ensure_built():
    lib = os.path.join(ROOT, "dist-lr_amd", "lib", "libdistlr_amd.so")
    orc = os.path.join(ROOT, "oracle", "build", "liblr_oracle.so")
    if not os.path.exists(orc):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "build/liblr_oracle.so"], check=True)
    if not os.path.exists(lib):
        subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "dist-lr_amd")], check=True)


_ensure_built()


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


def read_golden_json(name):
    import json
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)
