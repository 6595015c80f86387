"""Test configuration: GPU marker, import paths, and on-demand build of the two native libraries.

`-m gpu` tests need an MI355X (they call libsr_amd.so); everything else runs on CPU.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "symbolicregression.jl_amd")
for p in (ROOT, PKG, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def _lib_is_current():
    """libsr_amd.so was built from exactly these sources and compile flags: the hash its link rule
    wrote beside it (untracked, written only next to a library make actually linked) equals
    `make print-srchash` here (a GPU-box snapshot carries the library but no object files, so make
    alone would rebuild everything)."""
    stamp = os.path.join(PKG, "lib", "libsr_amd.so.srchash")
    if not (os.path.exists(stamp) and os.path.exists(os.path.join(PKG, "lib", "libsr_amd.so"))):
        return False
    try:
        want = subprocess.run(["make", "-s", "--no-print-directory", "-C", PKG, "print-srchash"], check=True,
                              capture_output=True, text=True).stdout.strip()
    except (FileNotFoundError, subprocess.CalledProcessError):
        return False
    with open(stamp) as fh:
        return bool(want) and fh.read().strip() == want


def _ensure_built():
    """Run the (incremental) builds unless the library provably matches the sources: a stale shipped
    .so must never stand in for HEAD's sources.  Where no compiler exists (a GPU box without hipcc
    never happens on this pool) the prebuilt libraries are used as they are."""
    builds = [(os.path.join(ROOT, "oracle"), "-j1")]
    if not _lib_is_current():
        builds.insert(0, (PKG, "-j8"))
    for d, jobs in builds:
        try:
            subprocess.run(["make", "-s", jobs, "-C", d], check=True)
        except FileNotFoundError:
            pass


_ensure_built()


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X GPU (runs libsr_amd kernels)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def golden():
    import json

    with open(os.path.join(ROOT, "tests", "golden", "reference_known_answers.json")) as f:
        return json.load(f)
