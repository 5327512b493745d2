"""PHBase host logic on CPU: slicing, node slots, and the full PH control flow
driven through a CPU stand-in batch, single rank and 2-rank gloo."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from oracle import models as om
from oracle.ph_oracle import OraclePH


def _opts(**kw):
    o = {"solvername": "mi355x_pdhg", "PHIterLimit": 6, "defaultPHrho": 1.0,
         "convthresh": 1e-9, "verbose": False, "display_progress": False,
         "display_timing": False, "iter0_solver_options": {}, "iterk_solver_options": {}}
    o.update(kw)
    return o


def _run_ph(opts, names, creator, kw=None, nodes=None, mpicomm=None):
    from mpisppy_amd.opt.ph import PH
    from cpu_batch import CPUBatch
    ph = PH(dict(opts), names, creator, all_nodenames=nodes, mpicomm=mpicomm,
            scenario_creator_kwargs=kw)
    ph.batch = CPUBatch(ph.batch_data)
    conv, eobj, tb = ph.ph_main()
    return ph, conv, eobj, tb


def test_spbase_slices_and_probabilities():
    from mpisppy_amd.opt.ph import PH
    from mpisppy_amd.examples import hydro
    names, nodes = hydro.all_names_and_nodes()
    ph = PH(_opts(branching_factors=[3, 3]), names, hydro.scenario_creator, all_nodenames=nodes,
            scenario_creator_kwargs={"branching_factors": [3, 3]})
    assert ph.G == 16                        # ROOT(4) + 3 x ROOT_b(4)
    pc = ph.prob_coeff_host
    assert np.allclose(pc[:4], 1 / 9) and np.allclose(pc[4:], 1 / 3)   # spbase.py:353-366
    assert list(ph.slot_s0_host[4:8]) == [0] * 4 and list(ph.slot_s1_host[4:8]) == [3] * 4
    assert list(ph.slot_s0_host[12:16]) == [6] * 4


def test_farmer_ph_host_flow_matches_oracle_single_rank():
    from mpisppy_amd.examples import farmer
    S = 6
    names = [f"scen{i}" for i in range(S)]
    ph, conv, eobj, tb = _run_ph(_opts(), names, farmer.scenario_creator)
    orc = OraclePH(_opts(), [om.farmer(n) for n in names])
    oc, oe, ot = orc.ph_main()
    assert abs(tb - ot) < 1e-9 * abs(ot)
    assert abs(eobj - oe) < 1e-9 * abs(oe)
    assert abs(conv - oc) < 1e-9 * abs(oc)
    W = ph.W.view(ph.K, ph.S_loc).numpy().T
    assert np.allclose(W, np.array(orc.W), rtol=1e-9, atol=1e-9)


def test_hydro_ph_host_flow_matches_oracle():
    from mpisppy_amd.examples import hydro
    names, nodes = hydro.all_names_and_nodes()
    opts = _opts(PHIterLimit=10, convthresh=1e-3, branching_factors=[3, 3])
    ph, conv, eobj, tb = _run_ph(opts, names, hydro.scenario_creator,
                                 kw={"branching_factors": [3, 3]}, nodes=nodes)
    orc = OraclePH(opts, [om.hydro(n) for n in names])
    oc, oe, ot = orc.ph_main()
    assert ph._PHIter == orc.iters
    assert abs(tb - ot) < 1e-8 * abs(ot)
    assert abs(eobj - oe) < 1e-8 * abs(oe)


def test_ref_n_proc_emulates_reference_rank_count():
    from mpisppy_amd.examples import farmer
    names = [f"scen{i}" for i in range(7)]
    ph, conv, _, _ = _run_ph(_opts(PHIterLimit=3, ref_n_proc=3), names, farmer.scenario_creator)
    orc = OraclePH(_opts(PHIterLimit=3), [om.farmer(n) for n in names], n_proc=3)
    oc, _, _ = orc.ph_main()
    assert abs(conv - oc) < 1e-9 * abs(oc)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "mpi-sppy_amd"), os.path.join(root, "tests")):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mpisppy_amd.examples import hydro
        names, nodes = hydro.all_names_and_nodes()
        opts = _opts(PHIterLimit=10, convthresh=1e-3, branching_factors=[3, 3])
        ph, conv, eobj, tb = _run_ph(opts, names, hydro.scenario_creator,
                                     kw={"branching_factors": [3, 3]}, nodes=nodes)
        q.put((rank, conv, eobj, tb, ph._PHIter, ph.local_scenario_names))
    finally:
        torch.distributed.destroy_process_group()


def test_two_rank_gloo_hydro_matches_oracle():
    """Scenarios split 4/5 over 2 ranks (the reference's slicing); per-node
    xbar sums, conv and bounds go through gloo allreduce."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    assert res[0][5] == [f"Scen{i}" for i in range(1, 5)]
    assert res[1][5] == [f"Scen{i}" for i in range(5, 10)]
    opts = _opts(PHIterLimit=10, convthresh=1e-3)
    orc = OraclePH(opts, [om.hydro(f"Scen{i + 1}") for i in range(9)], n_proc=2)
    oc, oe, ot = orc.ph_main()
    for rank, conv, eobj, tb, iters, _ in res:
        assert iters == orc.iters
        assert abs(conv - oc) < 1e-8 * abs(oc)
        assert abs(eobj - oe) < 1e-8 * abs(oe)
        assert abs(tb - ot) < 1e-8 * abs(ot)


def _farmer_worker(rank, world, port, q, convthresh):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "mpi-sppy_amd"), os.path.join(root, "tests")):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mpisppy_amd.examples import farmer
        names = [f"scen{i}" for i in range(30)]
        opts = _opts(PHIterLimit=40, convthresh=convthresh)
        ph, conv, eobj, tb = _run_ph(opts, names, farmer.scenario_creator)
        hist = ph.conv_hist[:ph._PHIter].cpu().numpy().tolist()
        q.put((rank, conv, eobj, tb, ph._PHIter, hist))
    finally:
        torch.distributed.destroy_process_group()


@pytest.mark.parametrize("convthresh", [1e-4, 1.0])
def test_two_rank_gloo_lagged_conv_matches_oracle(convthresh):
    """Several ranks: the conv partials ride in the next pass's xbar-sum
    allreduce (one collective per iteration).  At the limit (1e-4) and on a
    convergence break at iteration 25 (1.0: the speculative solve is undone)
    the iteration count, conv history, Eobj (evaluated at the stale x) and
    trivial bound equal the oracle on 2 reference ranks."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_farmer_worker, args=(r, 2, port, q, convthresh))
             for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    orc = OraclePH(_opts(PHIterLimit=40, convthresh=convthresh),
                   [om.farmer(f"scen{i}") for i in range(30)], n_proc=2)
    oc, oe, ot = orc.ph_main()
    assert orc.iters == (40 if convthresh < 1e-2 else 25)
    for rank, conv, eobj, tb, iters, hist in res:
        assert iters == orc.iters
        assert abs(conv - oc) < 1e-6 * abs(oc)
        assert abs(hist[-1] - oc) < 1e-6 * abs(oc)
        assert abs(eobj - oe) < 1e-7 * abs(oe)
        assert abs(tb - ot) < 1e-8 * abs(ot)


def test_wxbar_csv_round_trip_and_checks(tmp_path):
    """utils/wxbarutils: the reference's csv formats, round trip of W and
    xbar, missing-variable and dual-feasibility errors (wxbarutils.py:212-261)."""
    from mpisppy_amd.utils import wxbarutils as wx
    from mpisppy_amd.examples import farmer
    names = [f"scen{i}" for i in range(3)]
    ph, conv, eobj, tb = _run_ph(_opts(PHIterLimit=3), names, farmer.scenario_creator)
    wfile = tmp_path / "w.csv"
    xfile = tmp_path / "xbar.csv"
    wx.write_W_to_file(ph, str(wfile))
    wx.write_xbar_to_file(ph, str(xfile))
    wx.write_W_to_file(ph, str(tmp_path / "wdir"), sep_files=True)
    lines = wfile.read_text().strip().split("\n")
    assert len(lines) == 3 * ph.K and lines[0].startswith("scen0,DevotedAcreage[")
    W0 = ph.W.clone()
    xb0 = ph.xbar.clone()
    ph.W.zero_()
    ph.xbar.zero_()
    wx.set_W_from_file(str(wfile), ph, 0)
    assert torch.equal(ph.W, W0)
    ph.W.zero_()
    wx.set_W_from_file(str(tmp_path / "wdir"), ph, 0, sep_files=True)
    assert torch.equal(ph.W, W0)
    wx.set_xbar_from_file(str(xfile), ph)
    assert torch.allclose(ph.xbar, xb0, rtol=0, atol=0)
    assert torch.allclose(ph.xsqbar, xb0 * xb0)
    # comments are ignored; a non-zero sum_s p_s W_s is rejected
    bad = tmp_path / "bad.csv"
    txt = "# comment\n" + "\n".join(lines[:-1]) + "\n" + lines[-1].rsplit(",", 1)[0] + ",12345.0\n"
    bad.write_text(txt)
    with pytest.raises(RuntimeError, match="dual feasibility"):
        wx.set_W_from_file(str(bad), ph, 0)
    miss = tmp_path / "miss.csv"
    miss.write_text("\n".join(lines[:-1]) + "\n")
    with pytest.raises(RuntimeError, match="missing"):
        wx.set_W_from_file(str(miss), ph, 0)


def test_wxbar_writer_reader_extensions(tmp_path):
    """WXBarWriter writes after PH; WXBarReader loads the files before Iter0
    of a new PH (wxbarwriter.py / wxbarreader.py)."""
    from mpisppy_amd.opt.ph import PH
    from mpisppy_amd.utils.wxbarwriter import WXBarWriter
    from mpisppy_amd.utils.wxbarreader import WXBarReader
    from mpisppy_amd.examples import farmer
    from cpu_batch import CPUBatch
    names = [f"scen{i}" for i in range(3)]
    wf, xf = str(tmp_path / "w.csv"), str(tmp_path / "x.csv")
    ph = PH(_opts(PHIterLimit=3, W_fname=wf, Xbar_fname=xf), names, farmer.scenario_creator,
            PH_extensions=WXBarWriter)
    ph.batch = CPUBatch(ph.batch_data)
    ph.ph_main()
    ph2 = PH(_opts(PHIterLimit=3, init_W_fname=wf, init_Xbar_fname=xf), names,
             farmer.scenario_creator, PH_extensions=WXBarReader)
    ph2.batch = CPUBatch(ph2.batch_data)
    ph2.PH_Prep()
    assert torch.equal(ph2.W, ph.W)
    assert torch.equal(ph2.xbar, ph.xbar)


def test_xhat_try_one_matches_oracle():
    """extensions/xhatbase._try_one on the host flow (CPU stand-in batch):
    nonants of one scenario fixed in all, LPs solved, Eobjective == the
    oracle's restatement; nonants and bounds restored afterwards."""
    from mpisppy_amd.extensions.xhatbase import XhatBase, xhat_shuffle_inner_bound
    from mpisppy_amd.examples import farmer
    from oracle.ph_oracle import xhat_objective
    names = [f"scen{i}" for i in range(3)]
    ph, conv, eobj, tb = _run_ph(_opts(PHIterLimit=3), names, farmer.scenario_creator)
    x_before = ph.batch.x.clone()
    xb = XhatBase(ph)
    obj = xb._try_one({"ROOT": "scen1"})
    xn = x_before.view(ph.batch.n, 3)[list(ph.batch_data.nonant_cols), 1].numpy()
    ref = xhat_objective([om.farmer(nm) for nm in names], {"ROOT": xn})
    assert abs(obj - ref) <= 1e-9 * abs(ref)
    cols = list(ph.batch_data.nonant_cols)
    assert torch.equal(ph.batch.x.view(ph.batch.n, 3)[cols], x_before.view(ph.batch.n, 3)[cols])
    assert ph.batch._lu is not None and np.array_equal(ph.batch._lu[0], ph.batch_data.l)
    best, who = xhat_shuffle_inner_bound(ph, tries=3)
    from oracle.ef import solve_ef
    ef, _ = solve_ef([om.farmer(nm) for nm in names])
    assert best >= ef - 1e-6 * abs(ef) and who in names


def test_hub_with_lagrangian_and_xhat_spokes_closes_the_gap():
    """cylinders/hub.PHHub with an in-process Lagrangian (outer) and xhat
    shuffle (inner) spoke on farmer: valid bounds around the EF optimum and
    termination on the relative gap (hub.py:119-137, 430-466)."""
    from mpisppy_amd.opt.ph import PH
    from mpisppy_amd.phbase import PHBase
    from mpisppy_amd.cylinders.hub import PHHub
    from mpisppy_amd.cylinders.lagrangian_bounder import LagrangianOuterBound
    from mpisppy_amd.cylinders.xhatshufflelooper_bounder import XhatShuffleInnerBound
    from mpisppy_amd.examples import farmer
    from cpu_batch import CPUBatch
    from oracle.ef import solve_ef
    names = [f"scen{i}" for i in range(3)]

    def mk(cls, **kw):
        o = cls(_opts(PHIterLimit=50, convthresh=-1.0, **kw), names, farmer.scenario_creator)
        o.batch = CPUBatch(o.batch_data)
        return o

    hub_opt = mk(PH)
    lag = LagrangianOuterBound(mk(PHBase))
    xh = XhatShuffleInnerBound(mk(PHBase))
    hub = PHHub(hub_opt, [lag, xh], options={"rel_gap": 0.01}, sync_every=2)
    hub.main()
    hub.hub_finalize()
    ef, _ = solve_ef([om.farmer(nm) for nm in names])
    assert hub.BestOuterBound <= ef + 1e-6 * abs(ef) <= hub.BestInnerBound + 2e-6 * abs(ef)
    assert hub.compute_gap() <= 0.01
    assert hub_opt._PHIter < 50


def test_bound_solves_use_tight_tolerance():
    """post_solve_bound and the Lagrangian spoke solve at bound_pdhg_tol
    (default 1e-12) unless the caller's solver options set pdhg_tol; PH
    solves keep the iterk options (bound solves)."""
    from mpisppy_amd.examples import farmer
    names = [f"scen{i}" for i in range(6)]
    ph, conv, eobj, tb = _run_ph(_opts(PHIterLimit=3), names, farmer.scenario_creator)
    seen = []
    orig = ph.batch.solve

    def spy(*a, **kw):
        seen.append(kw.get("tol"))
        return orig(*a, **kw)

    ph.batch.solve = spy
    ph.post_solve_bound()
    ph.post_solve_bound(solver_options={"pdhg_tol": 1e-9})
    ph.PHoptions["bound_pdhg_tol"] = 1e-11
    ph.post_solve_bound()
    ph.solve_loop(solver_options=ph.PHoptions["iterk_solver_options"])
    assert seen == [1e-12, 1e-9, 1e-11, 1e-9]


def _vprob(S):
    """Slot 0 of even scenarios carries probability 2/S, of odd ones 0 (its
    W is masked); every slot still sums to 1 over the scenarios."""
    def variable_probability(scen, first_name=None):
        s = int(scen.name[4:])
        return [(first_name, 2.0 / S if s % 2 == 0 else 0.0)]
    return variable_probability


def test_variable_probability_matches_oracle():
    """spbase.py:369-400 / phbase.py:246-251: per-variable probabilities
    replace prob_coeff in Compute_Xbar and zero-probability nonants have W
    masked; host flow (CPU stand-in batch) against the oracle."""
    from mpisppy_amd.opt.ph import PH
    from mpisppy_amd.examples import farmer
    from cpu_batch import CPUBatch
    S = 6
    names = [f"scen{i}" for i in range(S)]
    probe = PH(_opts(), names, farmer.scenario_creator)
    first = probe.nonant_names()[0]
    opts = _opts(PHIterLimit=5, variable_probability_kwargs={"first_name": first},
                 do_not_check_variable_probabilities=False)
    ph = PH(dict(opts), names, farmer.scenario_creator, variable_probability=_vprob(S))
    ph.batch = CPUBatch(ph.batch_data)
    conv, eobj, tb = ph.ph_main()
    vp = {s: {0: (2.0 / S if s % 2 == 0 else 0.0)} for s in range(S)}
    orc = OraclePH(opts, [om.farmer(n) for n in names], variable_prob=vp)
    oc, oe, ot = orc.ph_main()
    W = ph.W.view(ph.K, ph.S_loc).numpy().T
    assert np.allclose(W, np.array(orc.W), rtol=1e-9, atol=1e-9)
    assert np.all(W[1::2, 0] == 0.0) and np.any(W[0::2, 0] != 0.0)
    xb = ph.xbar.view(ph.K, ph.S_loc)[:, 0].numpy()
    assert np.allclose(xb, orc.xbar[0], rtol=1e-9, atol=1e-9)
    assert abs(conv - oc) < 1e-9 * abs(oc) and abs(eobj - oe) < 1e-9 * abs(oe)
    v = ph.gather_var_values_to_rank0()
    assert v[("scen1", first)] is None and v[("scen0", first)] is not None
    assert ph.gather_var_values_to_rank0(get_zero_prob_values=True)[("scen1", first)] is not None
    # a setter whose probabilities do not sum to 1 is rejected when checked
    with pytest.raises(RuntimeError, match="do not sum to 1"):
        PH(dict(opts), names, farmer.scenario_creator,
           variable_probability=lambda sc, first_name=None: [(first_name, 0.5)])


def _farmer3_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "mpi-sppy_amd"), os.path.join(root, "tests")):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mpisppy_amd.examples import doc_farmer
        names = ["good", "average", "bad"]
        opts = _opts(PHIterLimit=5, defaultPHrho=10, convthresh=1e-7)
        ph, conv, eobj, tb = _run_ph(opts, names, doc_farmer.scenario_creator)
        v = ph.gather_var_values_to_rank0()
        q.put((rank, conv, eobj, tb, ph._PHIter, list(ph.local_scenario_names), v))
    finally:
        torch.distributed.destroy_process_group()


def test_three_rank_gloo_doc_farmer_config1():
    """BASELINE config 1 ("farmer 3-scenario PH on CPU via mpiexec -n 3",
    examples/run_all.py:80-83): the doc farmer on three gloo ranks, one
    scenario per rank (sputils.py:625-628), through the host flow with the
    CPU stand-in batch (the product solver needs the GPU): the published
    per-scenario nonants after 5 PH iterations (doc/src/examples.rst:323-334)
    and the oracle's conv / Eobj / trivial bound on 3 reference ranks."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_farmer3_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=300) for _ in procs), key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r[5] for r in res] == [["good"], ["average"], ["bad"]]
    opts = _opts(PHIterLimit=5, defaultPHrho=10, convthresh=1e-7)
    orc = OraclePH(opts, [om.doc_farmer(n) for n in ("good", "average", "bad")], n_proc=3)
    oc, oe, ot = orc.ph_main()
    for rank, conv, eobj, tb, iters, _, _ in res:
        assert iters == orc.iters == 5
        assert abs(conv - oc) < 1e-8 * abs(oc)
        assert abs(eobj - oe) < 1e-8 * abs(oe)
        assert abs(tb - ot) < 1e-8 * abs(ot)
    v = res[0][6]
    ref = {("good", "X[BEETS]"): 280.6489711937925, ("average", "X[WHEAT]"): 136.72037037055298,
           ("bad", "X[CORN]"): 85.26131687116226}
    for k, r in ref.items():
        assert abs(v[k] - r) / abs(r) < 1e-8, (k, v[k], r)


def test_bundle_assignment_matches_reference_slicing():
    """spbase.py:206-240: each rank's scenarios cut into bundles_per_rank
    contiguous slices range(int(i*avg), int((i+1)*avg)); too many bundles
    is an error."""
    from mpisppy_amd.bundles import assign_bundles
    from mpisppy_amd.utils.sputils import rank_slices
    names = [f"scen{i}" for i in range(11)]
    nb = assign_bundles(rank_slices(11, 2), names, 2)
    assert nb[0] == {0: ["scen0", "scen1"], 1: ["scen2", "scen3", "scen4"]}
    assert nb[1] == {0: ["scen5", "scen6", "scen7"], 1: ["scen8", "scen9", "scen10"]}
    with pytest.raises(RuntimeError, match="Not enough scenarios"):
        assign_bundles(rank_slices(11, 2), names, 6)


def test_bundle_layout_is_the_bundles_extensive_form():
    """Each bundle of the batched layout (bundles.BundleLayout: T blocks of
    the scenario pattern + chained nonanticipativity rows, an inert pad
    block for a short bundle) solved as an LP equals oracle/ef.py's EF of
    its scenarios (star nonanticipativity rows, sputils.py:246-383), both
    with the scenarios' probabilities: P_b x bound_b == EF value."""
    from mpisppy_amd.opt.ph import PH
    from mpisppy_amd.examples import farmer
    from oracle.ef import solve_ef
    import scipy.sparse as sp
    from oracle.solve import solve_scenario
    names = [f"scen{i}" for i in range(11)]
    ph = PH(_opts(bundles_per_rank=4), names, farmer.scenario_creator)
    bl = ph.bundle_layout
    assert bl.T == 3 and bl.Sb == 4
    assert [len(v.scen_list) for v in ph.local_subproblems.values()] == [2, 3, 3, 3]
    d = bl.data
    for b, (bname, bv) in enumerate(ph.local_subproblems.items()):
        A = sp.csr_matrix((d.vals[:, b], d.col_idx, d.row_ptr), shape=(d.m, d.n))
        x, y, feas = solve_scenario(d.c[:, b], None, A, d.rl[:, b], d.ru[:, b], d.l[:, b], d.u[:, b])
        assert feas
        val = bl.P[b] * (float(d.c[:, b] @ x) + float(d.const[b]))
        scens = [om.farmer(nm) for nm in bv.scen_list]
        for sc in scens:
            sc.prob = 1.0 / len(names)
        ef, _ = solve_ef(scens)
        assert abs(val - ef) <= 1e-9 * abs(ef), (b, val, ef)


@pytest.mark.parametrize("S,bpr", [(12, 4), (11, 3)])
def test_bundled_ph_host_flow_matches_oracle(S, bpr):
    """PH with bundles_per_rank (phbase.py:1273-1302, 803-862, 985-995) on
    the CPU stand-in: the bundle batch's PH terms gathered with p_s / P_b,
    its solution scattered to the scenarios; trivial bound (bundle EF
    values), W, x-bar, conv and Eobj against the oracle PH on the same
    bundles."""
    from mpisppy_amd.opt.ph import PH
    from mpisppy_amd.examples import farmer
    from cpu_batch import CPUBatch
    names = [f"scen{i}" for i in range(S)]
    opts = _opts(PHIterLimit=8, bundles_per_rank=bpr)
    ph = PH(dict(opts), names, farmer.scenario_creator)
    ph.batch = CPUBatch(ph.batch_data)
    ph._create_bundle_batch(None, batch_factory=CPUBatch)
    conv, eobj, tb = ph.ph_main()
    idx = {nm: i for i, nm in enumerate(names)}
    bundles = [[idx[nm] for nm in bv.scen_list] for bv in ph.local_subproblems.values()]
    orc = OraclePH(dict(opts), [om.farmer(n) for n in names], bundles=bundles)
    oc, oe, ot = orc.ph_main()
    assert ph._PHIter == orc.iters
    assert abs(tb - ot) < 1e-9 * abs(ot)
    assert abs(eobj - oe) < 1e-8 * abs(oe)
    assert abs(conv - oc) < 1e-7 * abs(oc)
    W = ph.W.view(ph.K, ph.S_loc).numpy().T
    assert np.allclose(W, np.array(orc.W), rtol=1e-7, atol=1e-7)
    # the bundles' trivial bound is at least the scenarios' (a bundle is a
    # relaxation of fewer nonanticipativity constraints dropped)
    orc1 = OraclePH(dict(opts), [om.farmer(n) for n in names])
    assert tb >= orc1.Iter0() - 1e-9 * abs(tb)


def test_bundled_hydro_multistage_matches_oracle():
    """Bundles across tree nodes (hydro, 9 scenarios in 2 bundles: the first
    holds ROOT_0's three scenarios and one of ROOT_1): the chained
    nonanticipativity rows are active only between blocks of the same node
    at each slot; trivial bound, Eobj and conv against the oracle's star EF
    bundles."""
    from mpisppy_amd.opt.ph import PH
    from mpisppy_amd.examples import hydro
    from cpu_batch import CPUBatch
    names, nodes = hydro.all_names_and_nodes()
    opts = _opts(PHIterLimit=10, convthresh=1e-3, branching_factors=[3, 3], bundles_per_rank=2)
    ph = PH(dict(opts), names, hydro.scenario_creator, all_nodenames=nodes,
            scenario_creator_kwargs={"branching_factors": [3, 3]})
    ph.batch = CPUBatch(ph.batch_data)
    ph._create_bundle_batch(None, batch_factory=CPUBatch)
    conv, eobj, tb = ph.ph_main()
    assert [len(v.scen_list) for v in ph.local_subproblems.values()] == [4, 5]
    bl = ph.bundle_layout
    K = ph.K
    # block 3 of bundle 0 is Scen4 (ROOT_1): ROOT slots linked, ROOT_0/ROOT_1 slots not
    lrl = bl.data.rl[bl.T * ph.batch_data.m:, 0].reshape(bl.T - 1, K)
    assert np.all(lrl[2, :4] == 0.0) and np.all(np.isinf(lrl[2, 4:]))
    assert np.all(lrl[1] == 0.0)
    orc = OraclePH(dict(opts), [om.hydro(nm) for nm in names], bundles=[[0, 1, 2, 3], [4, 5, 6, 7, 8]])
    oc, oe, ot = orc.ph_main()
    assert ph._PHIter == orc.iters
    assert abs(tb - ot) < 1e-9 * abs(ot)
    assert abs(eobj - oe) < 1e-7 * abs(oe)
    assert abs(conv - oc) < 1e-6 * abs(oc)


def test_bundle_multistage_fixed_nonant_links_to_node_reference():
    """A fixed multistage nonant inside a bundle (advisor r5): the reference
    links every unfixed variable to the node's first scenario in the bundle
    (sputils.py:350-364, ref_vars) and writes no row for a fixed one
    (nonant_for_fixed_vars=False), so the later scenarios of the node are
    tied to the reference scenario, not to the fixed value.  Hydro, the
    bundle Scen1..Scen4 (ROOT_0's three and one of ROOT_1) with Scen2's
    stage-2 Vol fixed at 0 (the old chain tied Scen3 to that value: bundle
    value 108.589 against the reference's 106.375): the bundle's LP equals the
    oracle's EF with the same fixing."""
    from mpisppy_amd.opt.ph import PH
    from mpisppy_amd.examples import hydro
    from mpisppy_amd.bundles import BundleLayout
    from mpisppy_amd.batch import BatchData
    from oracle.ef import solve_ef
    from oracle.solve import solve_scenario
    import scipy.sparse as sp
    names, nodes = hydro.all_names_and_nodes()
    opts = _opts(branching_factors=[3, 3])
    ph = PH(dict(opts), names, hydro.scenario_creator, all_nodenames=nodes,
            scenario_creator_kwargs={"branching_factors": [3, 3]})
    d0 = ph.batch_data
    col = list(d0.var_names).index("Vol[2]")
    assert col in set(d0.nonant_cols.tolist())
    l, u = d0.l.copy(), d0.u.copy()
    fix_val = 0.0
    l[col, 1] = u[col, 1] = fix_val
    d = BatchData(d0.names, d0.row_ptr, d0.col_idx, d0.vals, d0.c, d0.const, l, u, d0.rl, d0.ru,
                  d0.nonant_cols, d0.node_infos, d0.sense, prob=d0.prob, var_names=d0.var_names)
    bl = BundleLayout(d, [[0, 1, 2, 3], [4, 5, 6, 7, 8]], ph.local_prob, ph.gid_host, ["b0", "b1"])
    bd = bl.data
    A = sp.csr_matrix((bd.vals[:, 0], bd.col_idx, bd.row_ptr), shape=(bd.m, bd.n))
    x, y, feas = solve_scenario(bd.c[:, 0], None, A, bd.rl[:, 0], bd.ru[:, 0], bd.l[:, 0], bd.u[:, 0])
    assert feas
    val = bl.P[0] * (float(bd.c[:, 0] @ x) + float(bd.const[0]))
    scens = [om.hydro(nm) for nm in names[:4]]
    oc = scens[1].var_names.index("Vol[2]")
    scens[1].l = scens[1].l.copy()
    scens[1].u = scens[1].u.copy()
    scens[1].l[oc] = scens[1].u[oc] = fix_val
    for sc in scens:
        sc.prob = 1.0 / len(names)
    ef, xs = solve_ef(scens, nonant_for_fixed_vars=False)
    assert abs(val - ef) <= 1e-9 * max(1.0, abs(ef)), (val, ef)
    # Scen3 (block 2) follows Scen1 (the node's reference), not Scen2's fixed value
    n = d.n
    assert abs(x[2 * n + col] - x[0 * n + col]) <= 1e-9 * max(1.0, abs(x[col]))
    assert abs(x[1 * n + col] - fix_val) <= 1e-12
    assert abs(x[0 * n + col] - fix_val) > 1e-3   # (the fixing is binding: a different EF than the chain's)


@pytest.mark.parametrize("by", ["name", "vardata"])
def test_rho_setter_matches_oracle(by):
    """phbase.py:556-588: rho_setter(scenario) -> [(var, rho)]; the var given
    by nonant name (batched scenarios, no models) or by VarData of the
    scenario's model; the PH trajectory with per-slot rho equals the
    oracle's with the same rho."""
    from mpisppy_amd.opt.ph import PH
    from mpisppy_amd.examples import farmer
    from cpu_batch import CPUBatch
    names = [f"scen{i}" for i in range(6)]
    rho_of = {"WHEAT0": 0.5, "CORN0": 2.0, "SUGAR_BEETS0": 1.5}

    def setter(scen):
        if by == "name":
            return [(f"DevotedAcreage[{c}]", r) for c, r in rho_of.items()]
        return [(scen.DevotedAcreage[c], r) for c, r in rho_of.items()]

    opts = _opts(PHIterLimit=6, per_scenario_models=(by == "vardata"))
    ph = PH(dict(opts), names, farmer.scenario_creator, rho_setter=setter)
    ph.batch = CPUBatch(ph.batch_data)
    conv, eobj, tb = ph.ph_main()
    orc = OraclePH(dict(opts), [om.farmer(n) for n in names])
    order = ph.nonant_names()
    r = np.array([rho_of[nm.split("[")[1].rstrip("]")] for nm in order])
    orc.Iter0()
    orc.rho = [r.copy() for _ in names]
    orc.iterk_loop()
    oe = orc.Eobjective()
    assert ph._PHIter == orc.iters
    assert abs(eobj - oe) < 1e-8 * abs(oe)
    W = ph.W.view(ph.K, ph.S_loc).numpy().T
    assert np.allclose(W, np.array(orc.W), rtol=1e-8, atol=1e-8)
