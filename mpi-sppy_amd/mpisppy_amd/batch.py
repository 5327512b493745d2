"""Scenario-batched layout: host extraction and the device-resident batch.

Every local scenario is extracted once (its "standard repn") into one shared
sparsity pattern with per-scenario values stored scenario-fastest
(``v[i*S + s]``), the layout the C-ABI (include/phgpu.h) consumes.

Maximize models are turned into min form here (c -> -c), exactly the sign
convention of ``phbase.py:1206-1209`` (``objfct.expr -= ph_term``): the PH
terms are then always *added* in min form.
"""
import ctypes

import numpy as np
import torch

from . import _native


class NodeInfo:
    """Per-scenario tree path: [(node_name, cond_prob, nlen)] in stage order."""

    def __init__(self, nodes):
        self.nodes = [(str(a), float(b), int(c)) for a, b, c in nodes]

    def key(self):
        return tuple(self.nodes)


class BatchData:
    """Host-side batched arrays for the local scenarios (numpy, float64)."""

    def __init__(self, names, row_ptr, col_idx, vals, c, const, l, u, rl, ru,
                 nonant_cols, node_infos, sense, prob=None, var_names=None,
                 models=None):
        self.names = list(names)
        self.S = len(self.names)
        self.row_ptr = np.ascontiguousarray(row_ptr, dtype=np.int32)
        self.col_idx = np.ascontiguousarray(col_idx, dtype=np.int32)
        self.m = self.row_ptr.size - 1
        self.nnz = self.col_idx.size
        self.vals = np.ascontiguousarray(vals, dtype=np.float64).reshape(self.nnz, self.S)
        self.n = int(np.asarray(c).shape[0])
        self.c = np.ascontiguousarray(c, dtype=np.float64).reshape(self.n, self.S)
        self.const = np.asarray(const, dtype=np.float64).reshape(self.S)
        self.l = np.ascontiguousarray(l, dtype=np.float64).reshape(self.n, self.S)
        self.u = np.ascontiguousarray(u, dtype=np.float64).reshape(self.n, self.S)
        self.rl = np.ascontiguousarray(rl, dtype=np.float64).reshape(self.m, self.S)
        self.ru = np.ascontiguousarray(ru, dtype=np.float64).reshape(self.m, self.S)
        self.nonant_cols = np.ascontiguousarray(nonant_cols, dtype=np.int32)
        self.K = self.nonant_cols.size
        self.node_infos = list(node_infos)
        self.sense = sense
        self.prob = None if prob is None else np.asarray(prob, dtype=np.float64)
        self.var_names = var_names
        self.models = models
        self.validate()

    def validate(self):
        if np.any(self.l > self.u):
            raise ValueError("a variable has lb > ub")
        if np.any(self.rl > self.ru):
            raise ValueError("a constraint has lower > upper")
        for ni in self.node_infos:
            if sum(x[2] for x in ni.nodes) != self.K:
                raise ValueError("scenario node nonant lengths do not add up to K")
        if self.sense not in ("min", "max"):
            raise ValueError("sense must be 'min' or 'max'")


def _node_info_of(model):
    nl = getattr(model, "_mpisppy_node_list", None)
    if nl is None:
        raise RuntimeError(f"_mpisppy_node_list not found on scenario {getattr(model, 'name', '?')}")
    return nl


def from_models(names, models):
    """Extract per-scenario models (LinearModel or Pyomo via repn) into one batch.

    The union of the scenarios' sparsity patterns is used as the shared
    pattern (entries absent in a scenario are stored as 0).
    """
    from . import repn
    forms = [repn.standard_form(m) for m in models]
    n = forms[0]["A"].shape[1]
    m_ = forms[0]["A"].shape[0]
    sense = forms[0]["sense"]
    for f in forms:
        if f["A"].shape != (m_, n):
            raise ValueError("scenarios differ in the number of rows/columns; "
                             "the batched layout needs one shape")
        if f["sense"] != sense:
            raise RuntimeError("scenarios have mixed objective senses")
    A0 = forms[0]["A"]
    same = all(np.array_equal(f["A"].indptr, A0.indptr) and np.array_equal(f["A"].indices, A0.indices)
               for f in forms)
    if same:
        row_ptr, col_idx = A0.indptr, A0.indices
        vals = np.stack([f["A"].data for f in forms], axis=1)
    else:
        pat = sum((abs(f["A"]) > 0).astype(np.int8) for f in forms).tocsr()
        pat.sort_indices()
        row_ptr, col_idx = pat.indptr, pat.indices
        vals = np.zeros((pat.nnz, len(forms)))
        for s, f in enumerate(forms):
            A = f["A"].tocsr()
            for i in range(m_):
                lo, hi = row_ptr[i], row_ptr[i + 1]
                pos = {j: p for p, j in enumerate(col_idx[lo:hi], start=lo)}
                for p in range(A.indptr[i], A.indptr[i + 1]):
                    vals[pos[A.indices[p]], s] = A.data[p]
    sgn = 1.0 if sense == "min" else -1.0
    c = np.stack([sgn * f["c"] for f in forms], axis=1)
    const = np.array([sgn * f["const"] for f in forms])
    l = np.stack([f["l"] for f in forms], axis=1)
    u = np.stack([f["u"] for f in forms], axis=1)
    rl = np.stack([f["rl"] for f in forms], axis=1) if m_ else np.zeros((0, len(forms)))
    ru = np.stack([f["ru"] for f in forms], axis=1) if m_ else np.zeros((0, len(forms)))
    # nonants: concatenation over the node list of each node's vardata list
    nonant_cols = None
    node_infos = []
    for model in models:
        nl = _node_info_of(model)
        cols = []
        nodes = []
        for node in nl:
            vd = node.nonant_vardata_list
            cols.extend(repn.column_of(model, v) for v in vd)
            nodes.append((node.name, node.cond_prob, len(vd)))
        if nonant_cols is None:
            nonant_cols = cols
        elif cols != nonant_cols:
            raise ValueError("scenarios disagree on the nonant columns; the batched "
                             "layout needs the same nonant columns in every scenario")
        node_infos.append(NodeInfo(nodes))
    prob = None
    if all(hasattr(mdl, "_mpisppy_probability") for mdl in models):
        prob = [float(mdl._mpisppy_probability) for mdl in models]
    return BatchData(names, row_ptr, col_idx, vals, c, const, l, u, rl, ru,
                     np.asarray(nonant_cols), node_infos, sense, prob=prob,
                     var_names=forms[0]["var_names"], models=models)


class DeviceBatch:
    """The batch resident in HBM plus the libphgpu handle that solves it."""

    def __init__(self, data: BatchData, device=None, stream=None):
        _native.require_gpu()
        lib = _native.load()
        self.lib = lib
        self.data = data
        self.dev = torch.device("cuda", torch.cuda.current_device()) if device is None else device
        self.S, self.n, self.m, self.nnz, self.K = data.S, data.n, data.m, data.nnz, data.K
        self.stream = stream
        f64 = dict(dtype=torch.float64, device=self.dev)

        def up(a):
            return torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float64).to(self.dev)

        vals = up(data.vals)
        self.c = up(data.c)
        self.l = up(data.l)
        self.u = up(data.u)
        self.rl = up(data.rl) if self.m else torch.zeros(1, **f64)
        self.ru = up(data.ru) if self.m else torch.zeros(1, **f64)
        h = _native._c_ptr()
        # the torch stream the library's launches are ordered on (collectives
        # on the batch's tensors are queued on it too, phbase._allreduce)
        self.torch_stream = torch.cuda.current_stream(self.dev) if stream is None else stream
        sh = _native.stream_handle(stream)
        self._stream_handle = sh.value or 0
        _native.check(lib.ph_batch_create(h, self.S, self.n, self.m, self.nnz,
                                          data.row_ptr.ctypes.data_as(_native._c_ptr),
                                          data.col_idx.ctypes.data_as(_native._c_ptr),
                                          sh), "ph_batch_create")
        self.handle = h
        _native.check(lib.ph_batch_bind(h, _native.ptr(vals), _native.ptr(self.c),
                                        _native.ptr(self.l), _native.ptr(self.u),
                                        _native.ptr(self.rl), _native.ptr(self.ru)),
                      "ph_batch_bind")
        _native.check(lib.ph_batch_set_nonants(h, self.K, data.nonant_cols.ctypes.data_as(_native._c_ptr)),
                      "ph_batch_set_nonants")
        _native.check(lib.ph_batch_sync(h), "ph_batch_sync")
        del vals
        # iterates and outputs (scenario-fastest)
        self.x = torch.zeros(self.n * self.S, **f64)
        self.y = torch.zeros(max(self.m, 1) * self.S, **f64)
        self.omega = torch.zeros(self.S, **f64)
        i32 = dict(dtype=torch.int32, device=self.dev)
        self.status = torch.zeros(self.S, **i32)
        self.iters = torch.zeros(self.S, **i32)
        self.pobj = torch.zeros(self.S, **f64)
        self.dbound = torch.zeros(self.S, **f64)
        self.const = up(data.const)
        self._summary = np.zeros(5, dtype=np.int64)
        self.time_kernel = False  # record HIP events around each solve launch
        self._events = None
        self.event_log = []       # every (start, end) event pair recorded

    def solve(self, W, rho, xbar, w_on, prox_on, tol=1e-9, max_iters=200000,
              check_every=64, warm_start=True, reflection=1.0, polish=True):
        opts = _native.SolveOpts(float(tol), int(max_iters), int(check_every),
                                 1 if warm_start else 0, float(reflection), 1 if polish else 0)
        if self.time_kernel:
            stream = torch.cuda.current_stream(self.dev) if self.stream is None else self.stream
            self._events = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            self._events[0].record(stream)
            self.event_log.append(self._events)
        _native.check(self.lib.ph_pdhg_solve(
            self.handle, _native.ptr(W), _native.ptr(rho), _native.ptr(xbar),
            float(w_on), float(prox_on), _native.ptr(self.x), _native.ptr(self.y),
            _native.ptr(self.omega), _native.ptr(self.status), _native.ptr(self.iters),
            _native.ptr(self.pobj), _native.ptr(self.dbound), opts), "ph_pdhg_solve")
        if self.time_kernel:
            self._events[1].record(stream)

    def kernel_ms(self):
        """Duration of the last solve launch (HIP events on the batch's stream)."""
        if self._events is None:
            return None
        return self._events[0].elapsed_time(self._events[1])

    def set_timing(self, on):
        """Record HIP events around the active-set and PDHG kernels of every
        solve (library side, on the launch stream)."""
        _native.check(self.lib.ph_batch_set_timing(self.handle, 1 if on else 0),
                      "ph_batch_set_timing")

    def read_timing(self):
        """(solves, total ms of the active-set, polish and PDHG kernels); syncs."""
        return self.read_timing_full()[:4]

    def read_timing_full(self):
        """read_timing + (launches, total ms) of the mid-size path's PDHG phase
        kernel and of its polish phase kernel; syncs."""
        out = np.zeros(8)
        _native.check(self.lib.ph_batch_read_timing(self.handle, out.ctypes.data_as(_native._c_ptr)),
                      "ph_batch_read_timing")
        return (int(out[0]), float(out[1]), float(out[2]), float(out[3]),
                int(out[4]), float(out[5]), int(out[6]), float(out[7]))

    def kernel_ms_all(self):
        """Durations (ms) of every solve recorded in event_log (synchronises)."""
        if self.event_log:
            self.event_log[-1][1].synchronize()
        return [e0.elapsed_time(e1) for e0, e1 in self.event_log]

    def summary(self):
        """(not optimal, sum of PDHG iterations, max iterations, polished, cached)
        of the last solve; synchronises the stream (one 40-byte copy)."""
        _native.check(self.lib.ph_batch_solve_summary(
            self.handle, self._summary.ctypes.data_as(_native._c_ptr)), "ph_batch_solve_summary")
        return tuple(int(v) for v in self._summary)

    def set_bounds(self, l, u):
        """Column bounds of every scenario ([n][S] device tensors, copied)."""
        _native.check(self.lib.ph_batch_set_bounds(self.handle, _native.ptr(l), _native.ptr(u)),
                      "ph_batch_set_bounds")

    def set_stream(self, stream_handle):
        """Point the library's launches at another HIP stream (a raw handle)."""
        _native.check(self.lib.ph_batch_set_stream(self.handle, ctypes.c_void_p(stream_handle)),
                      "ph_batch_set_stream")

    @property
    def stream_handle(self):
        return self._stream_handle

    # ---- device-side iteration control (ph_loop_* in include/phgpu.h)
    def loop_reset(self, start_iter, iter_limit, convthresh):
        _native.check(self.lib.ph_loop_reset(self.handle, int(start_iter), int(iter_limit),
                                             float(convthresh)), "ph_loop_reset")

    def loop_enable(self, on):
        _native.check(self.lib.ph_loop_enable(self.handle, 1 if on else 0), "ph_loop_enable")

    def loop_set_xbar(self, prob_coeff, slot_k, slot_s0, slot_s1, out):
        """Let the post-solve kernel compute the next iteration's xbar sums."""
        G = 0 if slot_k is None else slot_k.numel()
        _native.check(self.lib.ph_loop_set_xbar(self.handle, _native.ptr(self.x),
                                                _native.ptr(prob_coeff), G, _native.ptr(slot_k),
                                                _native.ptr(slot_s0), _native.ptr(slot_s1),
                                                _native.ptr(out)), "ph_loop_set_xbar")

    def loop_conv_local(self, absdiff, seg, cnt, nproc, parts, conv_hist):
        _native.check(self.lib.ph_loop_conv_local(self.handle, _native.ptr(absdiff), _native.ptr(seg),
                                                  seg.numel() - 1, _native.ptr(cnt), float(nproc),
                                                  _native.ptr(parts), _native.ptr(conv_hist)),
                      "ph_loop_conv_local")

    def loop_update_w_conv(self, sums, G, gid, rho, w_coeff, xbar, xsqbar, W, absdiff, wconv,
                           conv_hist):
        _native.check(self.lib.ph_loop_update_w_conv(
            self.handle, _native.ptr(self.x), _native.ptr(sums), G, _native.ptr(gid),
            _native.ptr(rho), _native.ptr(w_coeff), _native.ptr(xbar), _native.ptr(xsqbar),
            _native.ptr(W), _native.ptr(absdiff), _native.ptr(wconv), _native.ptr(conv_hist)),
            "ph_loop_update_w_conv")

    def loop_conv(self, parts, cnt, nproc, conv_hist):
        _native.check(self.lib.ph_loop_conv(self.handle, _native.ptr(parts), _native.ptr(cnt),
                                            parts.numel(), float(nproc),
                                            _native.ptr(conv_hist)), "ph_loop_conv")

    def loop_conv_lagged(self, parts, cnt, nproc, conv_hist):
        _native.check(self.lib.ph_loop_conv_lagged(self.handle, _native.ptr(parts), _native.ptr(cnt),
                                                   parts.numel(), float(nproc),
                                                   _native.ptr(conv_hist)), "ph_loop_conv_lagged")

    def loop_backup(self, x_save, y_save):
        """Save x and y before this pass's solve (several-rank device loop)."""
        _native.check(self.lib.ph_loop_backup(self.handle, _native.ptr(self.x), _native.ptr(x_save),
                                              self.x.numel(), _native.ptr(self.y),
                                              _native.ptr(y_save), self.y.numel()),
                      "ph_loop_backup")

    def loop_backup_status(self, status_save, dbound_save):
        """Save the solve's status and outer bound with x/y (same stop check)."""
        _native.check(self.lib.ph_loop_backup_status(self.handle, _native.ptr(self.status),
                                                     _native.ptr(status_save),
                                                     _native.ptr(self.dbound),
                                                     _native.ptr(dbound_save)),
                      "ph_loop_backup_status")

    def loop_bind_pass(self, sums, G, gid, rho, w_coeff, xbar, xsqbar, W, absdiff, wconv,
                       conv_hist, conv_part, saves, w_on, prox_on, tol=1e-9,
                       max_iters=200000, check_every=64, warm_start=True, reflection=1.0,
                       polish=True):
        """Bind the arguments of ph_loop_pass for this loop (see phgpu.h);
        conv_part / saves = (x_save, y_save, status_save, dbound_save) on
        several ranks, None on one."""
        P = _native.ptr
        xs, ys, ss, ds = saves if saves is not None else (None, None, None, None)
        a = _native.LoopPassArgs(
            P(sums), int(G), P(gid), P(rho), P(w_coeff), P(xbar), P(xsqbar), P(W), P(absdiff),
            P(wconv), P(conv_hist), P(conv_part), P(xs), P(ys), P(ss), P(ds), float(w_on),
            float(prox_on), P(self.x), P(self.y), P(self.omega), P(self.status), P(self.iters),
            P(self.pobj), P(self.dbound),
            _native.SolveOpts(float(tol), int(max_iters), int(check_every),
                              1 if warm_start else 0, float(reflection), 1 if polish else 0))
        _native.check(self.lib.ph_loop_bind_pass(self.handle, ctypes.byref(a)), "ph_loop_bind_pass")

    def loop_unbind_pass(self):
        _native.check(self.lib.ph_loop_bind_pass(self.handle, None), "ph_loop_bind_pass")

    def loop_pass(self):
        """One device-loop pass (ph_loop_pass): one call per PH iteration."""
        _native.check(self.lib.ph_loop_pass(self.handle), "ph_loop_pass")

    def loop_run(self, iters):
        """Up to `iters` device-loop passes in one call (ph_loop_run): on one
        rank a persistent launch when the batch qualifies and PHGPU_PERSIST=1,
        else `iters` ph_loop_pass calls inside the library."""
        _native.check(self.lib.ph_loop_run(self.handle, int(iters)), "ph_loop_run")

    def loop_persistent(self):
        """True when loop_run takes the persistent path for the bound pass."""
        return bool(self.lib.ph_loop_persistent(self.handle))

    def loop_fused(self):
        """True when a loop_run since the last loop_reset ran the fused two-launch pass."""
        return bool(self.lib.ph_loop_fused(self.handle))

    def loop_read_timing(self):
        """(loop_kernel launches, their total ms, passes they ran) while timing."""
        out = np.zeros(3, dtype=np.float64)
        _native.check(self.lib.ph_loop_read_timing(self.handle, out.ctypes.data_as(_native._c_ptr)),
                      "ph_loop_read_timing")
        return float(out[0]), float(out[1]), int(out[2])

    def loop_status(self):
        """(stop, iter, not-optimal solves, solves, PDHG iters sum, max, polished,
        cached); synchronises.  stop: 0 running, 1 converged, 2 iteration limit."""
        out = np.zeros(8, dtype=np.int64)
        _native.check(self.lib.ph_loop_status(self.handle, out.ctypes.data_as(_native._c_ptr)),
                      "ph_loop_status")
        return tuple(int(v) for v in out)

    def xbar_accum(self, prob_coeff, slot_k, slot_s0, slot_s1, out):
        G = slot_k.numel()
        _native.check(self.lib.ph_xbar_accum(self.handle, _native.ptr(self.x), _native.ptr(prob_coeff),
                                             G, _native.ptr(slot_k), _native.ptr(slot_s0),
                                             _native.ptr(slot_s1), _native.ptr(out)), "ph_xbar_accum")

    def update_w(self, sums, G, gid, rho, w_coeff, xbar, xsqbar, W, absdiff):
        _native.check(self.lib.ph_update_w(self.handle, _native.ptr(self.x), _native.ptr(sums), G,
                                           _native.ptr(gid), _native.ptr(rho), _native.ptr(w_coeff),
                                           _native.ptr(xbar), _native.ptr(xsqbar), _native.ptr(W),
                                           _native.ptr(absdiff)), "ph_update_w")

    def segment_sum(self, v, w, seg, out):
        R = seg.numel() - 1
        _native.check(self.lib.ph_segment_sum(self.handle, _native.ptr(v), _native.ptr(w), R,
                                              _native.ptr(seg), _native.ptr(out)), "ph_segment_sum")

    def gather(self, src, idx, wt, count, dst):
        """dst[e] = wt[e] * src[idx[e]] on the batch's stream (ph_gather)."""
        _native.check(self.lib.ph_gather(self.handle, _native.ptr(src), int(src.numel()), _native.ptr(idx),
                                         _native.ptr(wt), int(count), _native.ptr(dst)), "ph_gather")

    def eval_objective(self, W, rho, xbar, w_on, prox_on, out):
        _native.check(self.lib.ph_eval_objective(self.handle, _native.ptr(self.x), _native.ptr(W),
                                                 _native.ptr(rho), _native.ptr(xbar), float(w_on),
                                                 float(prox_on), _native.ptr(out)), "ph_eval_objective")

    def diagnostics(self):
        """[S][5] host array: final (primal res, dual res, gap, fixed-point res,
        how: 0 PDHG tol, 1 warm-start polish, 2 polish of a PDHG iterate,
        3 active-set cache)."""
        out = np.zeros((self.S, _native.DIAG_W))
        _native.check(self.lib.ph_batch_get_diag(self.handle, out.ctypes.data_as(_native._c_ptr)),
                      "ph_batch_get_diag")
        return out

    def x_host(self):
        return self.x.view(self.n, self.S).cpu().numpy()

    def close(self):
        if getattr(self, "handle", None) is not None:
            self.lib.ph_batch_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
