"""CPU tests of the supernodal (multifrontal) analysis the big path's polish
uses on large KKT patterns (mpi-sppy_amd/csrc/kkt_super.h): the device plan
covers every supernode once per level with disjoint LDS shares, and a CPU
replay of the device's gather-form factorisation and solve
(tests/native/kkt_super_check.cpp, the algorithm of solve_super.inc) solves
a random quasi-definite KKT system of an active set to rounding error --
on farmer, sslp, random patterns and the UC LP relaxation's pattern
(N = 126,771, the pattern the per-entry factorisation could not take)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-sppy_amd"))
CSRC = os.path.join(ROOT, "mpi-sppy_amd", "csrc")
HARNESS = os.path.join(ROOT, "tests", "native", "kkt_super_check.cpp")


@pytest.fixture(scope="module")
def check_exe(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("ksup") / "kkt_super_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", CSRC, HARNESS, "-o", exe], check=True)
    return exe


def run(exe, n, m, row_ptr, col_idx, seed=1, ffix=0.2, finact=0.3, delta=0.5):
    inp = (f"{n} {m} {len(col_idx)}\n" + " ".join(map(str, row_ptr)) + "\n" + " ".join(map(str, col_idx)) +
           f"\n{seed} {ffix} {finact} {delta}\n")
    out = subprocess.run([exe], input=inp, capture_output=True, text=True, check=True).stdout
    return json.loads(out)


def farmer_pattern(c):
    from mpisppy_amd.examples import farmer
    from mpisppy_amd import batch
    names = ["scen0", "scen1"]
    d = batch.from_models(names, [farmer.scenario_creator(nm, crops_multiplier=c) for nm in names])
    return d.l.shape[0], d.m, d.row_ptr, d.col_idx


def random_pattern(rng, n, m, density):
    rows = []
    for i in range(m):
        cols = np.flatnonzero(rng.random(n) < density)
        if cols.size == 0:
            cols = np.array([rng.integers(n)])
        rows.append(np.sort(cols))
    row_ptr = np.concatenate([[0], np.cumsum([len(r) for r in rows])])
    return n, m, row_ptr, np.concatenate(rows)


def _check(d, N):
    assert "error" not in d, d
    assert d["N"] == N
    assert d["plan_ok"] == 1
    assert d["max_w"] <= 32 and d["max_f"] <= 1024
    # a quasi-definite system with delta = 0.5 is well conditioned: rounding error only
    assert d["residual"] <= 1e-11 * max(1.0, d["znorm"]), d


@pytest.mark.parametrize("c", [1, 10, 100])
def test_farmer_patterns(check_exe, c):
    n, m, rp, ci = farmer_pattern(c)
    d = run(check_exe, n, m, rp, ci, seed=c)
    _check(d, n + m)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_random_patterns(check_exe, seed):
    rng = np.random.default_rng(seed)
    n, m, rp, ci = random_pattern(rng, 300, 200, 0.02)
    d = run(check_exe, n, m, rp, ci, seed=seed, ffix=0.1 * seed, finact=0.2)
    _check(d, n + m)


def test_sslp_pattern(check_exe):
    from mpisppy_amd.examples import sslp
    from mpisppy_amd import batch
    names = sslp.scenario_names(5)[:2]
    d0 = batch.from_models(names, [sslp.scenario_creator(nm, data_dir="data/sslp_15_45_5/scenariodata")
                                   for nm in names])
    n = d0.l.shape[0]
    d = run(check_exe, n, d0.m, d0.row_ptr, d0.col_idx)
    _check(d, n + d0.m)


def test_uc_pattern(check_exe):
    """The UC LP relaxation's KKT: the supernodal form factors it with
    ~1.4e8 flops in 27 levels (the per-entry form needed 58M update gathers
    per factorisation); both a well-conditioned and the polish's delta =
    1e-7 system are solved (the latter to a relative residual)."""
    from mpisppy_amd.examples import uc
    d0 = uc.batch_creator(["Scenario1", "Scenario2"])
    n = d0.l.shape[0]
    d = run(check_exe, n, d0.m, d0.row_ptr, d0.col_idx)
    _check(d, n + d0.m)
    assert d["ncontrib"] > 50_000_000 and d["nlev"] <= 40
    # delta = 1e-7: |z| ~ 1e7, a backward-stable solve leaves |K z - b| at
    # rounding times |K| |z| (|K| ~ 10^2 here)
    d2 = run(check_exe, n, d0.m, d0.row_ptr, d0.col_idx, delta=1e-7)
    assert d2["residual"] <= 1e-9 * d2["znorm"], d2
