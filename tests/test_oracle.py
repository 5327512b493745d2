"""Pin the CPU oracle to the reference's own golden values (CPU, no GPU)."""
import math

import numpy as np
import pytest

from oracle import models as om
from oracle.ef import solve_ef
from oracle.ph_oracle import OraclePH, rank_slices
from oracle.solve import solve_scenario, kkt_residual


def round_pos_sig(x, sig=1):
    """mpisppy/tests/test_ef_ph.py:66-67."""
    return round(x, sig - int(math.floor(math.log10(abs(x)))) - 1)


def test_doc_farmer_deterministic_lp():
    # doc/src/examples.rst:98-113: average yields -> -118600.0
    s = om.doc_farmer("average")
    x, y, feas = solve_scenario(s.c, None, s.A, s.rl, s.ru, s.l, s.u)
    assert feas
    assert f"{s.c @ x:.1f}" == "-118600.0"


def test_doc_farmer_extensive_form():
    # doc/src/examples.rst:219-245: EF -108390.0, X = WHEAT 170, CORN 80, BEETS 250
    obj, xs = solve_ef([om.doc_farmer(n) for n in ["good", "average", "bad"]])
    assert f"{obj:.1f}" == "-108390.0"
    assert np.allclose(xs[0][:3], [170.0, 80.0, 250.0], atol=1e-7)


def test_doc_farmer_ph_published_nonants():
    # doc/src/examples.rst:253-265 (options) and :323-334 (values)
    opts = {"PHIterLimit": 5, "defaultPHrho": 10, "convthresh": 1e-7}
    scens = [om.doc_farmer(n) for n in ["good", "average", "bad"]]
    ph = OraclePH(opts, scens)
    ph.ph_main()
    ref = {"good": [280.6489711937925, 85.26131687116064, 134.0897119350402],
           "average": [283.2796296293019, 80.00000000014425, 136.72037037055298],
           "bad": [280.64897119379475, 85.26131687116226, 134.08971193504266]}
    for s, sc in enumerate(scens):
        got = ph.x[s][[2, 1, 0]]   # X[BEETS], X[CORN], X[WHEAT]
        assert np.allclose(got, ref[sc.name], rtol=1e-8, atol=0), (sc.name, got)


def test_hydro_reference_test_values():
    # mpisppy/tests/test_ef_ph.py:44-60 options, :541-559 asserted values
    scens = [om.hydro(f"Scen{i + 1}") for i in range(9)]
    ph = OraclePH({"PHIterLimit": 10, "defaultPHrho": 1, "convthresh": 0.001}, scens)
    conv, eobj, tb = ph.ph_main()
    assert round_pos_sig(tb, 2) == 180
    ph.w_on = ph.prox_on = 0.0
    assert round_pos_sig(ph.Eobjective(), 2) == 190


def test_hydro_ef_value():
    # mpisppy/tests/test_ef_ph.py:505-521: EF Scen7.Pgt[2] ~ 60 (1 s.f.)
    scens = [om.hydro(f"Scen{i + 1}") for i in range(9)]
    obj, xs = solve_ef(scens)
    assert round_pos_sig(xs[6][1], 1) == 60


def test_rank_slices_match_reference_formula():
    # sputils.py:625-628
    assert rank_slices(10, 3) == [[0, 1, 2], [3, 4, 5], [6, 7, 8, 9]]
    assert rank_slices(7, 1) == [list(range(7))]


def test_qp_polish_is_kkt_exact():
    scens = [om.farmer(f"scen{i}", 2) for i in range(4)]
    ph = OraclePH({"PHIterLimit": 1, "defaultPHrho": 1.0, "convthresh": 0}, scens)
    ph.Iter0()
    ph.Compute_Xbar(); ph.Update_W()
    for s in range(4):
        g, q, _ = ph._terms(s, 1.0, 1.0)
        sc = scens[s]
        x, y, feas = solve_scenario(g, q, sc.A, sc.rl, sc.ru, sc.l, sc.u)
        pv, dv = kkt_residual(x, y, g, q, sc.A, sc.rl, sc.ru, sc.l, sc.u)
        assert max(pv, dv) < 1e-9


def test_farmer_yields_restate_reference_rng():
    # farmer.py:54,150-156: seeded by scennum; rand() per crop in CROPS order for groupnum>0
    s = om.farmer("scen5", 2)
    rs = np.random.RandomState(5)
    expect = [3.0 + rs.rand(), 3.6 + rs.rand(), 24.0 + rs.rand(),
              3.0 + rs.rand(), 3.6 + rs.rand(), 24.0 + rs.rand()]   # scen5 -> AboveAverage1
    got = [-s.A[7 + k, k] for k in range(6)]    # LimitAmountSold rows carry -Yield*DA
    assert np.allclose(got, expect)
    assert om.farmer("scen1", 1).A[1, 0] == 2.5   # groupnum 0: base yield, no draw


def test_sslp_lp_relaxation_bounds():
    """sslp_15_45_5 LP relaxation (no reference pin exists for sslp: parity
    unpinned against the reference, checked for consistency here): the PH
    trivial bound is a valid lower bound of the EF, Eobj after 10 PH
    iterations is finite, and every prox-QP
    solve passes the KKT check (the oracle raises otherwise)."""
    from oracle.ef import solve_ef
    names = [f"Scenario{i + 1}" for i in range(5)]
    sc = [om.sslp(n, "sslp_15_45_5") for n in names]
    ef_val, _ = solve_ef(sc)
    orc = OraclePH({"PHIterLimit": 10, "defaultPHrho": 1.0, "convthresh": 1e-6}, sc)
    conv, eobj, tb = orc.ph_main()
    assert tb <= ef_val + 1e-9 * abs(ef_val)
    assert abs(ef_val - (-280.4902709111119)) < 1e-6
    assert abs(tb - (-291.989987012987)) < 1e-6
    assert orc.iters == 10 and 0.0 < conv < 0.05


def test_farmer_ef_golden_fixture_reproduces():
    # tests/golden/farmer_ef.json was written by tests/golden/make_golden.py;
    # the S=1000 case is re-solved here (the 10k case takes ~15 s)
    import json
    import os
    with open(os.path.join(os.path.dirname(__file__), "golden", "farmer_ef.json")) as f:
        gold = [g for g in json.load(f)["cases"] if g["S"] == 1000][0]
    scens = [om.farmer(f"scen{i}", 1, num_scens=1000) for i in range(1000)]
    obj, xs = solve_ef(scens)
    assert abs(obj - gold["ef_obj"]) <= 1e-9 * abs(obj)
    idx = scens[0].nodes[0][2]
    assert np.allclose([xs[0][i] for i in idx], gold["nonants"], rtol=1e-8)
    # every scenario shares the first stage (non-anticipativity rows)
    assert max(np.max(np.abs(x[idx] - xs[0][idx])) for x in xs) < 1e-7


def test_batched_oracle_pins_to_distributed_highs_oracle():
    """oracle/batch_pdas.py (batched exact active-set prox-QP solves, which
    generated tests/golden/farmer10k_ph.json) against oracle/ph_dist.py
    (HiGHS + KKT polish per subproblem on 6 gloo ranks, the `mpiexec -n 6`
    restatement): same farmer instance, rho 1, convthresh 1e-4, the
    reference's per-rank convergence metric for 6 ranks
    (tests/golden/farmer200_ph_dist.json).  The HiGHS path accepts QP points
    at 1e-9 relative KKT, the batched one is exact to ~1e-14, so values agree
    to ~1e-8 and the iteration count exactly."""
    import json
    import os
    from oracle.batch_pdas import ph_run
    with open(os.path.join(os.path.dirname(__file__), "golden", "farmer200_ph_dist.json")) as f:
        ref = json.load(f)
    scens = [om.farmer(f"scen{i}", 1) for i in range(ref["S"])]
    r = ph_run(scens, ref["rho"], ref["convthresh"], 100000, ref["ranks"])
    assert r["iterations"] == ref["iterations"]
    assert np.max(np.abs(np.array(r["xbar"]) - ref["xbar"]) / np.abs(ref["xbar"])) < 1e-7
    assert abs(r["Eobj"] - ref["Eobj"]) < 1e-9 * abs(ref["Eobj"])
    assert abs(r["trivial_bound"] - ref["trivial_bound"]) < 1e-12 * abs(ref["trivial_bound"])
    assert abs(float(np.abs(r["W"]).sum()) - ref["W_abs_sum"]) < 1e-7 * ref["W_abs_sum"]
    for k, w in ref["W_sample"].items():
        assert np.max(np.abs(r["W"][int(k)] - np.array(w))) < 1e-6 * max(1.0, np.max(np.abs(w)))


def test_farmer10k_golden_trajectory_fixture_is_consistent():
    """tests/golden/farmer10k_ph.json (oracle/batch_pdas.py, 10,000 scenarios,
    regenerated by `python -m oracle.batch_pdas --scens 10000`, ~25 min):
    conv below the threshold only at the last pass (the break of
    phbase.py:1505-1510), xbar within the acreage limit, bound below Eobj."""
    import json
    import os
    with open(os.path.join(os.path.dirname(__file__), "golden", "farmer10k_ph.json")) as f:
        g = json.load(f)
    assert g["S"] == 10000 and g["conv"] < g["convthresh"]
    assert g["conv_history_tail"][-2] >= g["convthresh"]       # the break is at the first pass below
    assert 0.0 <= sum(g["xbar"]) <= 500.0 * (1 + 1e-12)          # total acreage (farmer.py:183-186)
    assert g["trivial_bound"] < g["Eobj"]                       # minimisation: a lower bound
