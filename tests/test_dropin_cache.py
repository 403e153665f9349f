"""The drop-in's host bookkeeping (hb_mcmc_amd/csrc/hb_dropin.hpp) on the CPU:
exact light-curve cache (two light curves forced onto one hash key get two
contexts), logL memo by exact parameter bytes (one flipped bit is a fresh
evaluation), LRU eviction and the call combiner under 25 threads
(mcmc_wrapper2.c:383-489).  Built with g++ from tests/dropin_cache_test.cpp
against a fake context, so no GPU is needed."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_dropin_cache_memo_combiner(tmp_path):
    exe = str(tmp_path / "dropin_cache_test")
    src = os.path.join(ROOT, "tests", "dropin_cache_test.cpp")
    b = subprocess.run(["g++", "-O1", "-std=c++17", "-Wall", "-pthread", "-o", exe, src], capture_output=True,
                       text=True)
    assert b.returncode == 0, b.stderr[-3000:]
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip().splitlines()[-1] == "ok", r.stdout[-2000:] + r.stderr[-2000:]
