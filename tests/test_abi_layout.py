"""C-ABI library: loads, exports every symbol of include/phgpu.h, validates
arguments without a GPU; product layout builders agree with the oracle's
independent restatement of the reference models."""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_functions():
    txt = open(os.path.join(ROOT, "include", "phgpu.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(ph_[a-z_]+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    from mpisppy_amd import _native
    lib = _native.load()
    funcs = _header_functions()
    assert len(funcs) >= 12
    for f in funcs:
        assert hasattr(lib, f), f
    declared = {name for name, _, _ in _native.SIGNATURES}
    assert declared == set(funcs)
    assert lib.ph_version().decode().startswith("phgpu")


def test_invalid_arguments_fail_before_touching_the_gpu():
    from mpisppy_amd import _native
    lib = _native.load()
    h = ctypes.c_void_p()
    rp = np.array([0, 1], dtype=np.int32)
    ci = np.array([5], dtype=np.int32)   # column out of range for n=2
    rc = lib.ph_batch_create(h, 1, 2, 1, 1, rp.ctypes.data_as(ctypes.c_void_p),
                             ci.ctypes.data_as(ctypes.c_void_p), None)
    assert rc == -1
    assert b"col_idx" in lib.ph_last_error()
    rc = lib.ph_batch_create(h, 0, 2, 1, 1, rp.ctypes.data_as(ctypes.c_void_p),
                             ci.ctypes.data_as(ctypes.c_void_p), None)
    assert rc == -1
    assert lib.ph_pdhg_solve(None, None, None, None, 0.0, 0.0, None, None, None, None,
                             None, None, None, None) == -1


def test_solver_requires_gpu_or_raises():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from mpisppy_amd.opt.ph import PH
    from mpisppy_amd.examples import farmer
    opts = {"solvername": "mi355x_pdhg", "PHIterLimit": 1, "defaultPHrho": 1.0,
            "convthresh": 0.0, "verbose": False, "display_progress": False,
            "iter0_solver_options": {}, "iterk_solver_options": {}}
    ph = PH(opts, ["scen0", "scen1"], farmer.scenario_creator)
    with pytest.raises(RuntimeError, match="GPU"):
        ph.ph_main()


def test_unknown_solvername_rejected():
    from mpisppy_amd.opt.ph import PH
    from mpisppy_amd.examples import farmer
    opts = {"solvername": "gurobi_persistent", "PHIterLimit": 1, "defaultPHrho": 1.0,
            "convthresh": 0.0, "verbose": False, "display_progress": False,
            "iter0_solver_options": {}, "iterk_solver_options": {}}
    with pytest.raises(ValueError):
        PH(opts, ["scen0"], farmer.scenario_creator)


def _dense(bd, s):
    import scipy.sparse as sp
    return sp.csr_matrix((bd.vals[:, s], bd.col_idx, bd.row_ptr), shape=(bd.m, bd.n)).toarray()


@pytest.mark.parametrize("c", [1, 3])
def test_farmer_layout_matches_oracle_models(c):
    from mpisppy_amd.examples import farmer
    from mpisppy_amd.batch import from_models
    from oracle import models as om
    names = [f"scen{i}" for i in range(7)]
    bd = farmer.batch_creator(names, crops_multiplier=c)
    bm = from_models(names, [farmer.scenario_creator(n, crops_multiplier=c) for n in names])
    for k in ("row_ptr", "col_idx", "vals", "c", "l", "u", "rl", "ru", "nonant_cols"):
        assert np.array_equal(getattr(bd, k), getattr(bm, k)), k
    for s, nm in enumerate(names):
        o = om.farmer(nm, c)
        assert np.array_equal(_dense(bd, s), o.A.toarray())
        assert np.array_equal(bd.c[:, s], o.c)
        assert np.array_equal(bd.rl[:, s], o.rl) and np.array_equal(bd.ru[:, s], o.ru)
        assert np.array_equal(bd.u[:, s], o.u)
        assert list(bd.nonant_cols) == list(o.nonant_idx)


def test_farmer_maximize_sense_is_negated_into_min_form():
    from mpisppy_amd.examples import farmer
    from mpisppy_amd.batch import from_models
    names = ["scen0", "scen4"]
    bmin = from_models(names, [farmer.scenario_creator(n) for n in names])
    bmax = from_models(names, [farmer.scenario_creator(n, sense="max") for n in names])
    assert bmax.sense == "max"
    assert np.array_equal(bmin.c, bmax.c)


def test_hydro_and_doc_farmer_layout_match_oracle():
    from mpisppy_amd.examples import hydro, doc_farmer
    from mpisppy_amd.batch import from_models
    from oracle import models as om
    names = [f"Scen{i + 1}" for i in range(9)]
    bd = from_models(names, [hydro.scenario_creator(n, [3, 3]) for n in names])
    for s, nm in enumerate(names):
        o = om.hydro(nm)
        assert np.allclose(_dense(bd, s), o.A.toarray(), rtol=0, atol=0)
        assert np.array_equal(bd.rl[:, s], o.rl) and np.array_equal(bd.ru[:, s], o.ru)
        assert np.array_equal(bd.l[:, s], o.l) and np.array_equal(bd.u[:, s], o.u)
        assert list(bd.nonant_cols) == list(o.nonant_idx)
        assert [n[0] for n in bd.node_infos[s].nodes] == [n[0] for n in o.nodes]
    names = ["good", "average", "bad"]
    bd = from_models(names, [doc_farmer.scenario_creator(n) for n in names])
    for s, nm in enumerate(names):
        o = om.doc_farmer(nm)
        assert np.array_equal(_dense(bd, s), o.A.toarray())
        assert list(bd.nonant_cols) == list(o.nonant_idx)


@pytest.mark.parametrize("inst", ["sslp_15_45_5", "sslp_5_25_50", "sslp_15_45_synthetic"])
def test_sslp_layout_matches_oracle(inst):
    """sslp LP relaxation: the batch builder, the per-scenario LinearModel
    path and the oracle restatement give the same arrays."""
    import scipy.sparse as sp
    from mpisppy_amd.batch import from_models
    from mpisppy_amd.examples import sslp
    from oracle import models as om
    names = sslp.scenario_names(4)
    bd = sslp.batch_creator(names, instance=inst)
    md = from_models(names, [sslp.scenario_creator(nm, instance=inst) for nm in names])
    for a in ["row_ptr", "col_idx", "vals", "c", "l", "u", "rl", "ru", "nonant_cols"]:
        assert np.array_equal(getattr(bd, a), getattr(md, a)), a
    for s, nm in enumerate(names):
        o = om.sslp(nm, inst)
        A = sp.csr_matrix((bd.vals[:, s], bd.col_idx, bd.row_ptr), shape=(bd.m, bd.n)).toarray()
        assert np.array_equal(A, o.A.toarray())
        assert np.array_equal(bd.c[:, s], o.c)
        assert np.array_equal(bd.rl[:, s], o.rl) and np.array_equal(bd.ru[:, s], o.ru)
        assert np.array_equal(bd.l[:, s], o.l) and np.array_equal(bd.u[:, s], o.u)
        assert list(bd.nonant_cols) == list(o.nonant_idx)
    # data_dir form of the reference's scenario_creator (sslp.py:17-25)
    m = sslp.scenario_creator("Scenario1", data_dir=f"data/{inst}/scenariodata")
    assert m.num_vars == bd.n


def test_ctypes_structs_match_the_header_layout(tmp_path):
    """The ctypes mirrors of ph_solve_opts and ph_loop_pass_args have the C
    compiler's size and field offsets (gcc on include/phgpu.h)."""
    import shutil
    import subprocess
    from mpisppy_amd import _native
    if shutil.which("gcc") is None:
        pytest.skip("no gcc")
    structs = {"ph_solve_opts": _native.SolveOpts, "ph_loop_pass_args": _native.LoopPassArgs}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "phgpu.h"', "int main(void) {"]
    for cname, cls in structs.items():
        lines.append(f'  printf("{cname} size %zu\\n", sizeof({cname}));')
        for fname, _ in cls._fields_:
            lines.append(f'  printf("{cname} {fname} %zu\\n", offsetof({cname}, {fname}));')
    lines += ["  return 0;", "}"]
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines) + "\n")
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), "-o", str(exe), str(src)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    got = {(a, b): int(c) for a, b, c in (ln.split() for ln in out if ln)}
    for cname, cls in structs.items():
        assert got[(cname, "size")] == ctypes.sizeof(cls), cname
        for fname, _ in cls._fields_:
            assert got[(cname, fname)] == getattr(cls, fname).offset, (cname, fname)


def test_uc_layout_matches_oracle():
    """BASELINE config 4's model (examples/uc.py: ReferenceModel_OK.py's LP
    relaxation on the WECC-240 data) against the oracle's independent
    restatement (oracle/models.py uc): the same shape, nonants (UnitOn in
    sorted key order) and, per scenario wind, the same LP optimum (HiGHS on
    both); the batch carries each scenario's wind bounds."""
    import scipy.sparse as sp
    from mpisppy_amd.examples import uc
    from oracle import models as om
    from oracle.solve import _highs_solve
    names = ["Scenario1", "Scenario7"]
    bd = uc.batch_creator(names)
    assert (bd.n, bd.m, bd.K) == (56869, 69902, 4080)
    for s, nm in enumerate(names):
        sc = om.uc(nm)
        assert sc.A.shape == (bd.m, bd.n)
        assert len(sc.nonant_idx) == bd.K
        A = sp.csr_matrix((bd.vals[:, s], bd.col_idx, bd.row_ptr), shape=(bd.m, bd.n))
        st1, x1, _, _ = _highs_solve(bd.c[:, s], None, A, bd.rl[:, s], bd.ru[:, s], bd.l[:, s], bd.u[:, s],
                                     time_limit=120)
        st2, x2, _, _ = _highs_solve(sc.c, None, sc.A, sc.rl, sc.ru, sc.l, sc.u, time_limit=120)
        v1 = float(bd.c[:, s] @ x1 + bd.const[s])
        v2 = float(sc.c @ x2)
        assert abs(v1 - v2) <= 1e-9 * abs(v2), (nm, v1, v2)
        # nonant values of two exact vertices need not agree (degenerate LP);
        # the nonant names are UnitOn in sorted (generator, period) order
    nn = [bd.var_names[j] for j in bd.nonant_cols]
    assert nn[0] == "UnitOn[('BRIDGER_20_6333_C', 1)]" and nn[1] == "UnitOn[('BRIDGER_20_6333_C', 2)]"
    rhos = dict(uc.scenario_rhos(None))
    assert len(rhos) == bd.K and min(rhos.values()) >= 0.0
