"""CPU tests of the host symbolic analysis the mid-size and big polish
kernels rely on (mpi-sppy_amd/csrc/kkt_symbolic.h): the level-ordered
numbering (the device reads level l's columns and entries as contiguous
ranges), the fill pattern, and the device's level-scheduled factorisation
and solve replayed in numpy against a dense LDL' of the same permuted
quasi-definite KKT matrix."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-sppy_amd"))
CSRC = os.path.join(ROOT, "mpi-sppy_amd", "csrc")
HARNESS = os.path.join(ROOT, "tests", "native", "kkt_symbolic_dump.cpp")


@pytest.fixture(scope="module")
def dump_exe(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("kkt") / "kkt_symbolic_dump")
    subprocess.run(["g++", "-O1", "-std=c++17", "-I", CSRC, HARNESS, "-o", exe], check=True)
    return exe


def analyze(exe, n, m, row_ptr, col_idx):
    inp = f"{n} {m} {len(col_idx)}\n" + " ".join(map(str, row_ptr)) + "\n" + " ".join(map(str, col_idx)) + "\n"
    out = subprocess.run([exe], input=inp, capture_output=True, text=True, check=True).stdout
    d = json.loads(out)
    return {k: (np.asarray(v) if isinstance(v, list) else v) for k, v in d.items()}


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


def kkt_matrix(rng, n, m, row_ptr, col_idx, delta=1e-3):
    """A random quasi-definite [H -A'; -A -G] with the pattern's A."""
    N = n + m
    K = np.zeros((N, N))
    K[np.arange(n), np.arange(n)] = rng.uniform(0.5, 2.0, n) + delta
    K[n + np.arange(m), n + np.arange(m)] = -(rng.uniform(0.5, 2.0, m) + delta)
    vals = rng.uniform(-2.0, 2.0, len(col_idx))
    for i in range(m):
        for p in range(row_ptr[i], row_ptr[i + 1]):
            K[n + i, col_idx[p]] = K[col_idx[p], n + i] = -vals[p]
    return K, vals


def device_factor(sym, n, m, K, row_ptr, col_idx, vals):
    """The level-scheduled LDL' of polish_mid (solve_mid.inc), in numpy:
    Lv from the scatter of -A at apos, D from the diagonal, then per level
    the column pivots and the entries' updates from the ec lists."""
    N = n + m
    pos = sym["pos"]
    Dv = np.zeros(N)
    Dv[pos] = np.diag(K)
    Lv = np.zeros(sym["nnzL"])
    for p in range(len(col_idx)):
        Lv[sym["apos"][p]] = -vals[p]
    Lrp, Lrc, Lrq, lvp, lep = sym["Lrp"], sym["Lrc"], sym["Lrq"], sym["lvp"], sym["lep"]
    ecp, ec1, ec2, eck, Lcl = sym["ecp"], sym["ec1"], sym["ec2"], sym["eck"], sym["Lcl"]
    for lv in range(sym["NL"]):
        for c in range(lvp[lv], lvp[lv + 1]):  # level-ordered numbering: the columns
            d = Dv[c]
            for t in range(Lrp[c], Lrp[c + 1]):
                d -= Lv[Lrq[t]] ** 2 * Dv[Lrc[t]]
            Dv[c] = d
        for p in range(lep[lv], lep[lv + 1]):  # ... and their CSC entries
            v = Lv[p]
            for t in range(ecp[p], ecp[p + 1]):
                v -= Lv[ec1[t]] * Dv[eck[t]] * Lv[ec2[t]]
            Lv[p] = v / Dv[Lcl[p]]
    return Lv, Dv


def device_solve(sym, Lv, Dv, r):
    """kkt_ldl_solve's forward / backward sweeps over the level order."""
    w = r.copy()
    Lrp, Lrc, Lrq, Lcp, Lri = sym["Lrp"], sym["Lrc"], sym["Lrq"], sym["Lcp"], sym["Lri"]
    N = len(w)
    for c in range(N):
        w[c] -= sum(Lv[Lrq[t]] * w[Lrc[t]] for t in range(Lrp[c], Lrp[c + 1]))
    for c in range(N - 1, -1, -1):
        w[c] = w[c] / Dv[c] - sum(Lv[p] * w[Lri[p]] for p in range(Lcp[c], Lcp[c + 1]))
    return w


def check(exe, n, m, row_ptr, col_idx, seed):
    sym = analyze(exe, n, m, row_ptr, col_idx)
    assert "error" not in sym
    N = n + m
    assert sym["N"] == N
    # level-ordered numbering: lvc and lee are the identity, levels ascend
    assert np.array_equal(sym["lvc"], np.arange(N))
    assert np.array_equal(sym["lee"], np.arange(sym["nnzL"]))
    lvp = sym["lvp"]
    assert lvp[0] == 0 and lvp[-1] == N and np.all(np.diff(lvp) > 0)
    assert np.array_equal(sym["lep"], sym["Lcp"][lvp])
    # the top chain: one column per level from chain0 on
    assert np.all(np.diff(lvp)[sym["chain0"]:] == 1)
    # pos is a permutation; every L entry is strictly below its column
    assert np.array_equal(np.sort(sym["pos"]), np.arange(N))
    assert np.all(sym["Lri"] > sym["Lcl"])
    rng = np.random.default_rng(seed)
    K, vals = kkt_matrix(rng, n, m, row_ptr, col_idx)
    P = np.zeros((N, N))
    P[sym["pos"], np.arange(N)] = 1.0  # (P K P')[pos[u], pos[v]] = K[u, v]
    Kp = P @ K @ P.T
    # dense LDL' without pivoting (the permuted matrix is quasi-definite)
    L = np.eye(N)
    D = np.zeros(N)
    A = Kp.copy()
    for c in range(N):
        D[c] = A[c, c]
        L[c + 1:, c] = A[c + 1:, c] / D[c]
        A[c + 1:, c + 1:] -= np.outer(L[c + 1:, c], L[c + 1:, c]) * D[c]
    # the symbolic pattern holds every nonzero of L
    pat = np.zeros((N, N), dtype=bool)
    pat[sym["Lri"], sym["Lcl"]] = True
    off = np.abs(np.tril(L, -1)) > 1e-12
    assert not np.any(off & ~pat)
    Lv, Dv = device_factor(sym, n, m, K, row_ptr, col_idx, vals)
    np.testing.assert_allclose(Dv, D, rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(Lv, L[sym["Lri"], sym["Lcl"]], rtol=1e-10, atol=1e-12)
    b = rng.standard_normal(N)
    z = device_solve(sym, Lv, Dv, b)
    np.testing.assert_allclose(Kp @ z, b, rtol=1e-9, atol=1e-9)


@pytest.mark.parametrize("c", [1, 2, 5])
def test_farmer_symbolic_and_level_scheduled_factorisation(dump_exe, c):
    n, m, row_ptr, col_idx = farmer_pattern(c)
    check(dump_exe, n, m, row_ptr, col_idx, seed=c)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_random_pattern_symbolic_and_level_scheduled_factorisation(dump_exe, seed):
    rng = np.random.default_rng(100 + seed)
    n, m, row_ptr, col_idx = random_pattern(rng, 30, 20, 0.12)
    check(dump_exe, n, m, row_ptr, col_idx, seed=seed)


def test_farmer_c100_fill_is_the_mid_plan(dump_exe):
    """F3's KKT: the fill the DESIGN's LDS plan quotes (nnzL 3,001, 10
    levels, 901 update terms) fits the uint16 staged arrays."""
    n, m, row_ptr, col_idx = farmer_pattern(100)
    sym = analyze(dump_exe, n, m, row_ptr, col_idx)
    assert (sym["N"], sym["nnzL"], sym["NL"], sym["ncontrib"]) == (2101, 3001, 10, 901)
    assert sym["N"] < 65536 and sym["nnzL"] < 65535 and sym["ncontrib"] < 65535
