// phgpu.hip -- MI355X (gfx950) kernels + C-ABI for the batched PH hot path.
//
// Design:
//  * one workgroup owns one scenario for a whole PDHG solve; the scenario's
//    scaled matrix values, the current dual vector and the primal trial
//    point live in LDS; every thread owns CPT columns and RPT rows whose
//    state (x, anchor, objective, bounds, A x) lives in VGPRs;
//  * one PDHG step = a column phase (SpMV^T through the CSC view of the
//    shared pattern + primal prox step) and a row phase (SpMV through the
//    CSR view + dual prox step), two workgroup barriers, no HBM traffic;
//  * reflected Halpern iteration with adaptive restarts and primal-weight
//    updates (r2HPDHG), KKT/restart checks every `check_every` steps with
//    wave-shuffle + LDS block reductions;
//  * the nonanticipativity kernels (xbar sums, W update, convergence sums)
//    stream the scenario-fastest [k][s] arrays with coalesced FP64 loads.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/phgpu.h"

#define PHGPU_VERSION "phgpu 0.1 gfx950"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &msg) {
  g_err = msg;
  return code;
}

#define HIP_OK(expr)                                                        \
  do {                                                                      \
    hipError_t e_ = (expr);                                                 \
    if (e_ != hipSuccess)                                                   \
      return fail(PH_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

constexpr int WAVE = 64;
constexpr int MAX_WAVES = 16;  // 1024-thread blocks

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, WAVE);
  return v;
}

// Block-wide sum of NV values.  `red` is LDS scratch of MAX_WAVES*NV doubles.
// All threads receive the totals.  Contains two barriers.
template <int NV>
__device__ __forceinline__ void block_sum(double (&v)[NV], double *red) {
  const int lane = threadIdx.x & (WAVE - 1);
  const int wid = threadIdx.x / WAVE;
  const int nw = (blockDim.x + WAVE - 1) / WAVE;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    double t = wave_sum(v[i]);
    if (lane == 0) red[wid * NV + i] = t;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    double t = 0.0;
    for (int w = 0; w < nw; ++w) t += red[w * NV + i];
    v[i] = t;
  }
  __syncthreads();
}

__device__ __forceinline__ double clampd(double v, double lo, double hi) {
  return fmin(fmax(v, lo), hi);
}

struct Pattern {
  const int32_t *row_ptr;  // [m+1]
  const int32_t *col_idx;  // [nnz]
  const int32_t *col_ptr;  // [n+1]
  const int32_t *csc_row;  // [nnz]
  const int32_t *csc_k;    // [nnz]  CSR position of CSC entry
};

// Entries per line held in registers by the line's owner; longer lines are
// cut into extra chunks of LINE_D (see LineRegs).
constexpr int LINE_D = 4;

struct Chunks {
  int xr, xc;              // number of extra row / column chunks
  const int32_t *r_pb;     // [m+1] row i's partials are [r_pb[i], r_pb[i+1])
  const int32_t *r_pos;    // [xr] CSR position of the chunk's first entry
  const int32_t *r_len;    // [xr] entries in the chunk (<= LINE_D)
  const int32_t *c_pb;     // [n+1]
  const int32_t *c_pos;    // [xc] CSC position
  const int32_t *c_len;    // [xc]
};

// ------------------------------------------------------------------------
// Scaling kernel: per scenario Ruiz (10 sweeps) + Pock-Chambolle(alpha=1),
// writes dr [S][m], dc [S][n], scaled values [S][nnz] and the step size
// eta[s] = 0.995 / min(1, 1.02 * ||A~||_2 estimate) (||A~||_2 <= 1 after PC).
// ------------------------------------------------------------------------
template <int BLOCK, int CPT, int RPT>
__global__ void __launch_bounds__(BLOCK) scale_kernel(
    int S, int n, int m, int nnz, Pattern P, const double *__restrict__ vals,
    double *__restrict__ vals_s, double *__restrict__ dr_out,
    double *__restrict__ dc_out, double *__restrict__ eta_out) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int s = blockIdx.x;
  const int T = blockDim.x;
  const int tid = threadIdx.x;
  double *av = lds;            // [nnz] working |values|
  double *rsc = av + nnz;      // [m]
  double *csc = rsc + m;       // [n]
  double *vec = csc + n;       // [n] power iteration vector
  double *wv = vec + n;        // [m]
  double *red = wv + m;        // reduction scratch

  for (int k = tid; k < nnz; k += T) av[k] = vals[(size_t)k * S + s];
  for (int i = tid; i < m; i += T) rsc[i] = 1.0;
  for (int j = tid; j < n; j += T) csc[j] = 1.0;
  __syncthreads();

  for (int sweep = 0; sweep < 11; ++sweep) {
    const bool pc = (sweep == 10);  // last sweep: Pock-Chambolle (l1 norms)
    // row factors
    double rf[RPT];
#pragma unroll
    for (int b = 0; b < RPT; ++b) {
      int i = tid + b * T;
      rf[b] = 1.0;
      if (i < m) {
        double acc = 0.0;
        for (int p = P.row_ptr[i]; p < P.row_ptr[i + 1]; ++p) {
          double a = fabs(av[p]) * rsc[i] * csc[P.col_idx[p]];
          acc = pc ? acc + a : fmax(acc, a);
        }
        rf[b] = acc > 0.0 ? 1.0 / sqrt(acc) : 1.0;
      }
    }
    double cf[CPT];
#pragma unroll
    for (int b = 0; b < CPT; ++b) {
      int j = tid + b * T;
      cf[b] = 1.0;
      if (j < n) {
        double acc = 0.0;
        for (int p = P.col_ptr[j]; p < P.col_ptr[j + 1]; ++p) {
          int i = P.csc_row[p];
          double a = fabs(av[P.csc_k[p]]) * rsc[i] * csc[j];
          acc = pc ? acc + a : fmax(acc, a);
        }
        cf[b] = acc > 0.0 ? 1.0 / sqrt(acc) : 1.0;
      }
    }
    __syncthreads();
#pragma unroll
    for (int b = 0; b < RPT; ++b) {
      int i = tid + b * T;
      if (i < m) rsc[i] *= rf[b];
    }
#pragma unroll
    for (int b = 0; b < CPT; ++b) {
      int j = tid + b * T;
      if (j < n) csc[j] *= cf[b];
    }
    __syncthreads();
  }
  // scaled values
  for (int i = tid; i < m; i += T) {
    for (int p = P.row_ptr[i]; p < P.row_ptr[i + 1]; ++p)
      av[p] = av[p] * rsc[i] * csc[P.col_idx[p]];
  }
  for (int j = tid; j < n; j += T) vec[j] = 1.0;
  __syncthreads();
  // power iteration on A~^T A~
  double est = 1.0;
  for (int it = 0; it < 64; ++it) {
    for (int i = tid; i < m; i += T) {
      double acc = 0.0;
      for (int p = P.row_ptr[i]; p < P.row_ptr[i + 1]; ++p) acc += av[p] * vec[P.col_idx[p]];
      wv[i] = acc;
    }
    __syncthreads();
    double nv[1] = {0.0};
    double tv[CPT];
#pragma unroll
    for (int b = 0; b < CPT; ++b) {
      int j = tid + b * T;
      tv[b] = 0.0;
      if (j < n) {
        double acc = 0.0;
        for (int p = P.col_ptr[j]; p < P.col_ptr[j + 1]; ++p) acc += av[P.csc_k[p]] * wv[P.csc_row[p]];
        tv[b] = acc;
        nv[0] += acc * acc;
      }
    }
    block_sum<1>(nv, red);
    double nrm = sqrt(nv[0]);
    est = sqrt(nrm);  // ||A^T A v|| with ||v||=1 -> sigma_max^2 estimate
#pragma unroll
    for (int b = 0; b < CPT; ++b) {
      int j = tid + b * T;
      if (j < n) vec[j] = nrm > 0.0 ? tv[b] / nrm : 0.0;
    }
    __syncthreads();
  }
  for (int k = tid; k < nnz; k += T) vals_s[(size_t)s * nnz + k] = av[k];
  for (int i = tid; i < m; i += T) dr_out[(size_t)s * m + i] = rsc[i];
  for (int j = tid; j < n; j += T) dc_out[(size_t)s * n + j] = csc[j];
  if (tid == 0) {
    double sn = fmin(1.0, 1.02 * est);
    if (!(sn > 1e-12)) sn = 1.0;
    eta_out[s] = 0.995 / sn;
  }
}

struct SolveArgs {
  int S, n, m, nnz;
  Pattern P;
  Chunks X;
  const double *vals_s, *dr, *dc, *eta;
  const double *c, *l, *u, *rl, *ru;
  const int32_t *slot_of_col;
  const double *W, *rho, *xbar;
  double w_on, prox_on;
  double *x, *y, *omega;
  int32_t *status, *iters;
  double *pobj, *dbound;
  double *diag;  // [S][PH_DIAG_W]: final ep, ed, eg, r, how (library-owned)
  unsigned long long *summary;  // [4]: not optimal, sum iters, max iters, polished
  double tol;
  int max_iters, check_every, warm;
  double refl;
  int polish;  // 1: one-wave scenario with n + m <= POLISH_MAX and polish enabled
};

// Active-set polish: largest KKT system (free columns + active rows) and the
// KKT error below which a PDHG trial point is polished.
constexpr int POLISH_MAX = 63;
constexpr double POLISH_START = 1e-4;
constexpr int POLISH_ROUNDS = 6;

// Matrix entries a thread keeps in VGPRs for the lines (rows or columns) it
// owns plus the extra chunks of long lines it helps with.  A line's first
// LINE_D entries belong to its owner; entries beyond that are cut into
// chunks of LINE_D, numbered globally, spread over the block (chunk q is
// slot q / T of thread q % T) and summed into LDS partials part[q].  The
// owner adds its line's partials [pb, pb+pn).  Padded entries carry value 0
// and index 0, so every dot product is a fixed LINE_D-term unrolled FMA chain.
template <int P, int E>
struct LineRegs {
  int idx[P][LINE_D];
  double val[P][LINE_D];
  int pb[P], pn[P];
  int xidx[E > 0 ? E : 1][LINE_D];
  double xval[E > 0 ? E : 1][LINE_D];
  bool xon[E > 0 ? E : 1];

  // own line `line` (or nothing when line >= nlines); entries at pattern
  // positions [beg, end); entry p has index ix[p] and value v[vk ? vk[p] : p]
  __device__ __forceinline__ void load_own(int b, int line, int nlines, const int32_t *ptr,
                                           const int32_t *ix, const int32_t *vk,
                                           const double *v, const int32_t *xpb) {
    pb[b] = 0;
    pn[b] = 0;
    int beg = 0, len = 0;
    if (line < nlines) {
      beg = ptr[line];
      len = ptr[line + 1] - beg;
      if (xpb) {
        pb[b] = xpb[line];
        pn[b] = xpb[line + 1] - pb[b];
      }
    }
#pragma unroll
    for (int e = 0; e < LINE_D; ++e) {
      idx[b][e] = 0;
      val[b][e] = 0.0;
      if (e < len) {
        const int p = beg + e;
        idx[b][e] = ix[p];
        val[b][e] = v[vk ? vk[p] : p];
      }
    }
  }
  __device__ __forceinline__ void load_extra(int e, int q, int nx, const int32_t *xpos,
                                             const int32_t *xlen, const int32_t *ix,
                                             const int32_t *vk, const double *v) {
    xon[e] = q < nx;
    int beg = 0, len = 0;
    if (xon[e]) {
      beg = xpos[q];
      len = xlen[q];
    }
#pragma unroll
    for (int d = 0; d < LINE_D; ++d) {
      xidx[e][d] = 0;
      xval[e][d] = 0.0;
      if (d < len) {
        const int p = beg + d;
        xidx[e][d] = ix[p];
        xval[e][d] = v[vk ? vk[p] : p];
      }
    }
  }
  // out[b] = (line b of the matrix) . vec for every owned line.  Contains one
  // block barrier when E > 0 (partials), none otherwise; vec must be complete
  // in LDS before the call and part[] is free to overwrite.
  __device__ __forceinline__ void dots(const double *vec, double *part, double (&out)[P]) {
    if constexpr (E > 0) {
      const int T = blockDim.x;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        if (xon[e]) {
          double acc = 0.0;
#pragma unroll
          for (int d = 0; d < LINE_D; ++d) acc = fma(xval[e][d], vec[xidx[e][d]], acc);
          part[threadIdx.x + e * T] = acc;
        }
      }
      __syncthreads();
    }
#pragma unroll
    for (int b = 0; b < P; ++b) {
      double acc = 0.0;
#pragma unroll
      for (int d = 0; d < LINE_D; ++d) acc = fma(val[b][d], vec[idx[b][d]], acc);
      if constexpr (E > 0) {
        for (int q = pb[b]; q < pb[b] + pn[b]; ++q) acc += part[q];
      }
      out[b] = acc;
    }
  }
};

// ------------------------------------------------------------------------
// PDHG solve kernel: one workgroup per scenario, everything on chip.
// P = columns and rows owned per thread, E = extra chunk slots per thread.
// ------------------------------------------------------------------------
template <int BLOCK, int P, int E>
__global__ void __launch_bounds__(BLOCK) pdhg_kernel(SolveArgs a) {
  constexpr int CPT = P, RPT = P;
  constexpr bool POL = (BLOCK == WAVE && P == 1);  // polish needs lane == line
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int s = blockIdx.x;
  const int T = blockDim.x;
  const int tid = threadIdx.x;
  const int S = a.S, n = a.n, m = a.m;
  double *xs = lds;                 // [n]   primal trial point x^+ (shared)
  double *ys = xs + n;              // [m]   dual iterate / dual trial (shared)
  double *part_c = ys + m;          // [xc]  column-chunk partials
  double *part_r = part_c + a.X.xc; // [xr]  row-chunk partials
  double *red = part_r + a.X.xr;    // reduction scratch [MAX_WAVES*10]

  const double *vs = a.vals_s + (size_t)s * a.nnz;
  LineRegs<P, E> CL, RW;  // columns (CSC view), rows (CSR view)
#pragma unroll
  for (int b = 0; b < P; ++b) {
    CL.load_own(b, tid + b * T, n, a.P.col_ptr, a.P.csc_row, a.P.csc_k, vs, a.X.xc ? a.X.c_pb : nullptr);
    RW.load_own(b, tid + b * T, m, a.P.row_ptr, a.P.col_idx, nullptr, vs, a.X.xr ? a.X.r_pb : nullptr);
  }
#pragma unroll
  for (int e = 0; e < (E > 0 ? E : 0); ++e) {
    CL.load_extra(e, tid + e * T, a.X.xc, a.X.c_pos, a.X.c_len, a.P.csc_row, a.P.csc_k, vs);
    RW.load_extra(e, tid + e * T, a.X.xr, a.X.r_pos, a.X.r_len, a.P.col_idx, nullptr, vs);
  }
  double DOT[P];

  // ---- column state in registers
  double X[CPT], Z0X[CPT], G[CPT], Q[CPT], L[CPT], U[CPT], DC[CPT], XN[CPT];
  double cst = 0.0, gsq = 0.0;
#pragma unroll
  for (int b = 0; b < CPT; ++b) {
    int j = tid + b * T;
    X[b] = Z0X[b] = G[b] = Q[b] = XN[b] = 0.0;
    L[b] = U[b] = 0.0;
    DC[b] = 1.0;
    if (j < n) {
      double dcj = a.dc[(size_t)s * n + j];
      double g = a.c[(size_t)j * S + s], q = 0.0;
      int k = a.slot_of_col ? a.slot_of_col[j] : -1;
      if (k >= 0) {
        double W = a.W[(size_t)k * S + s], r = a.rho[(size_t)k * S + s];
        double xb = a.xbar[(size_t)k * S + s];
        g += a.w_on * W - a.prox_on * r * xb;
        q = a.prox_on * r;
        cst += a.prox_on * 0.5 * r * xb * xb;
      }
      DC[b] = dcj;
      G[b] = g * dcj;
      Q[b] = q * dcj * dcj;
      L[b] = a.l[(size_t)j * S + s] / dcj;
      U[b] = a.u[(size_t)j * S + s] / dcj;
      double x0 = a.warm ? a.x[(size_t)j * S + s] / dcj : 0.0;
      X[b] = clampd(x0, L[b], U[b]);
      Z0X[b] = X[b];
      gsq += G[b] * G[b];
    }
  }
  // ---- row state in registers
  double Y[RPT], Z0Y[RPT], AX[RPT], AZ0[RPT], RL[RPT], RU[RPT], DR[RPT];
  double YN[RPT], AXN[RPT];
  double bsq = 0.0;
#pragma unroll
  for (int b = 0; b < RPT; ++b) {
    int i = tid + b * T;
    Y[b] = Z0Y[b] = AX[b] = AZ0[b] = RL[b] = RU[b] = YN[b] = AXN[b] = 0.0;
    DR[b] = 1.0;
    if (i < m) {
      double d = a.dr[(size_t)s * m + i];
      DR[b] = d;
      RL[b] = a.rl[(size_t)i * S + s] * d;
      RU[b] = a.ru[(size_t)i * S + s] * d;
      Y[b] = a.warm ? a.y[(size_t)i * S + s] / d : 0.0;
      // keep the dual iterate sign-feasible for the row's bounds
      if (!isfinite(RL[b])) Y[b] = fmin(Y[b], 0.0);
      if (!isfinite(RU[b])) Y[b] = fmax(Y[b], 0.0);
      Z0Y[b] = Y[b];
      double bl = isfinite(RL[b]) ? RL[b] : 0.0;
      double bu = isfinite(RU[b]) ? RU[b] : 0.0;
      bsq += bl * bl + (isfinite(RL[b]) ? 0.0 : bu * bu);
    }
  }
  // initial primal weight, objective constant
  double omega, omega0;
  {
    double v[3] = {cst, gsq, bsq};
    block_sum<3>(v, red);
    cst = v[0];
    double gn = sqrt(v[1]), bn = sqrt(v[2]);
    omega0 = (gn > 1e-10 && bn > 1e-10) ? gn / bn : 1.0;
    omega = omega0;
    // warm primal weight, kept within 100x of the data-based weight: carried
    // unclamped across PH iterations it drifts (1e6x seen on farmer) into a
    // regime where FP64 round-off stalls the iteration above 1e-9.
    if (a.warm && a.omega[s] > 0.0) omega = clampd(a.omega[s], omega0 * 1e-2, omega0 * 1e2);
  }
  const double eta = a.eta[s];
  const double gam = a.refl;

  // A x for the starting point; ys <- y
#pragma unroll
  for (int b = 0; b < CPT; ++b) {
    int j = tid + b * T;
    if (j < n) xs[j] = X[b];
  }
#pragma unroll
  for (int b = 0; b < RPT; ++b) {
    int i = tid + b * T;
    if (i < m) ys[i] = Y[b];
  }
  __syncthreads();
  RW.dots(xs, part_r, DOT);
#pragma unroll
  for (int b = 0; b < RPT; ++b) {
    int i = tid + b * T;
    if (i < m) AX[b] = AZ0[b] = DOT[b];
  }
  __syncthreads();

  int k = 0;  // iterations since last restart
  int it = 0;
  int stat = PH_STATUS_ITERLIMIT;
  double r_restart = -1.0, r_prev = -1.0;
  double out_pobj = 0.0, out_dobj = 0.0;
  double d_ep = -1.0, d_ed = -1.0, d_eg = -1.0, d_r = -1.0;
  const int maxit = a.max_iters;
  int maxit_eff = maxit;
  const int chk = a.check_every > 0 ? a.check_every : 64;

  // step sizes change only with the primal weight: no FP64 division in the
  // iteration except the Halpern weight 1/(k+2)
  double tau = 0.0, sig = 0.0, IQ[CPT];
  auto set_steps = [&]() {
    tau = eta / omega;
    sig = eta * omega;
#pragma unroll
    for (int b = 0; b < CPT; ++b) IQ[b] = 1.0 / (1.0 + tau * Q[b]);
  };
  set_steps();

  double LAM[CPT];  // scaled reduced costs of the last KKT evaluation
  int how = 0;      // 0: PDHG reached tol, 1: polished at start, 2: polished mid-solve

  // Local KKT terms of the trial point (XN, YN, AXN), unscaled; ys must hold
  // YN.  v[0..5] = primal residual^2, dual residual^2, primal objective,
  // dual objective, |b|^2, |g|^2.  Contains the column products' barrier.
  auto kkt_local = [&](double (&v)[10]) {
    double pr2 = 0.0, dr2 = 0.0, po = 0.0, dob = 0.0, bl2 = 0.0, g2 = 0.0;
    CL.dots(ys, part_c, DOT);
#pragma unroll
    for (int b = 0; b < CPT; ++b) {
      int j = tid + b * T;
      LAM[b] = 0.0;
      if (j < n) {
        LAM[b] = Q[b] * XN[b] + G[b] - DOT[b];
        double lam = LAM[b] / DC[b];  // unscaled reduced cost
        double xu = XN[b] * DC[b];
        double lu = L[b] * DC[b], uu = U[b] * DC[b];
        double lp = isfinite(lu) ? fmax(lam, 0.0) : 0.0;
        double lm = isfinite(uu) ? fmin(lam, 0.0) : 0.0;
        double rd = lam - lp - lm;
        dr2 += rd * rd;
        double qx = Q[b] / (DC[b] * DC[b]);
        double gu = G[b] / DC[b];
        po += 0.5 * qx * xu * xu + gu * xu;
        dob += -0.5 * qx * xu * xu + (lp > 0.0 ? lp * lu : 0.0) + (lm < 0.0 ? lm * uu : 0.0);
        g2 += gu * gu;
      }
    }
#pragma unroll
    for (int b = 0; b < RPT; ++b) {
      int i = tid + b * T;
      if (i < m) {
        double axu = AXN[b] / DR[b];
        double rlu = RL[b] / DR[b], ruu = RU[b] / DR[b];
        double rp = axu - clampd(axu, rlu, ruu);
        pr2 += rp * rp;
        double yu = YN[b] * DR[b];
        dob += (yu > 0.0 ? yu * rlu : 0.0) + (yu < 0.0 ? yu * ruu : 0.0);
        if (isfinite(rlu)) bl2 += rlu * rlu;
      }
    }
    v[0] = pr2; v[1] = dr2; v[2] = po; v[3] = dob; v[4] = bl2; v[5] = g2;
  };
  // relative primal residual, dual residual and gap from block-summed terms;
  // records the objectives and the diagnostics
  auto kkt_measures = [&](const double (&v)[10], double &ep, double &ed, double &eg) {
    ep = sqrt(v[0]) / (1.0 + sqrt(v[4]));
    ed = sqrt(v[1]) / (1.0 + sqrt(v[5]));
    const double P0 = v[2] + cst, D0 = v[3] + cst;
    eg = fabs(P0 - D0) / (1.0 + fabs(P0) + fabs(D0));
    out_pobj = P0;
    out_dobj = D0;
    d_ep = ep; d_ed = ed; d_eg = eg;
  };

  // Active-set polish (one-wave scenarios, n + m <= POLISH_MAX; lane t owns
  // column t and row t).  A primal-dual active-set iteration on the exact
  // KKT system:
  //  1. classify the trial point: column at a bound when it lies within th
  //     (relative) of it, row active when its multiplier is nonzero beyond
  //     th relative to the largest one (|y| > th*max|y|);
  //  2. solve  q_F x_F - A_RF' y_R = -g_F,  A_RF x_F = b_R - A_R,fixed x_fixed
  //     by Gauss-Jordan elimination with partial pivoting in LDS (lane =
  //     matrix column); dependent columns (degenerate duplicate constraints,
  //     e.g. a row that repeats a variable bound) get the value 0;
  //  3. accept the clipped point when the full KKT check passes at a.tol,
  //     else re-classify by the primal-dual active-set rule
  //       at lower  <=>  lambda + (l - x) > 0,   row at rl <=> y + (rl - Ax) > 0
  //     and repeat (at most `rounds` solves, stopping on a repeated set).
  // On success XN/YN/AXN hold the exact point; on failure they are restored.
  unsigned long long pol_first[4] = {~0ull, ~0ull, ~0ull, ~0ull};
  auto polish_run = [&](double th, int rounds) -> bool {
    if constexpr (!POL) {
      return false;
    } else {
      const int lane = tid;
      const double sx = XN[0], sy = YN[0], sa = AXN[0], sl = LAM[0];
      double *kkt = red + MAX_WAVES * 10;
      int *cpos = (int *)(kkt + (size_t)(n + m) * (n + m + 1));
      // ---- 1. initial classification
      double sc_y = (lane < m) ? fabs(YN[0]) : 0.0;
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) sc_y = fmax(sc_y, __shfl_xor(sc_y, off, WAVE));
      int cs = 0;  // 0 free, 1 at L, 2 at U
      if (lane < n) {
        const double xv = XN[0];
        if (L[0] == U[0]) cs = 1;
        else if (isfinite(L[0]) && xv - L[0] <= th * (1.0 + fabs(L[0]))) cs = 1;
        else if (isfinite(U[0]) && U[0] - xv <= th * (1.0 + fabs(U[0]))) cs = 2;
      }
      int rs = 0;  // 0 inactive, 1 at rl, 2 at ru
      if (lane < m) {
        if (RL[0] == RU[0]) rs = 1;
        else if (isfinite(RL[0]) && YN[0] > th * sc_y) rs = 1;
        else if (isfinite(RU[0]) && YN[0] < -th * sc_y) rs = 2;
      }
      {
        const unsigned long long m0 = __ballot(cs == 1), m1 = __ballot(cs == 2);
        const unsigned long long m2 = __ballot(rs == 1), m3 = __ballot(rs == 2);
        if (m0 == pol_first[0] && m1 == pol_first[1] && m2 == pol_first[2] && m3 == pol_first[3])
          return false;  // this starting set was tried already
        pol_first[0] = m0; pol_first[1] = m1; pol_first[2] = m2; pol_first[3] = m3;
      }
      unsigned long long prev[4] = {~0ull, ~0ull, ~0ull, ~0ull};
      const unsigned long long below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
      for (int round = 0; round < rounds; ++round) {
        const unsigned long long m0 = __ballot(cs == 1), m1 = __ballot(cs == 2);
        const unsigned long long m2 = __ballot(rs == 1), m3 = __ballot(rs == 2);
        if (m0 == prev[0] && m1 == prev[1] && m2 == prev[2] && m3 == prev[3]) break;  // cycle
        prev[0] = m0; prev[1] = m1; prev[2] = m2; prev[3] = m3;
        // ---- 2. KKT system of the active set
        const bool fr = lane < n && cs == 0;
        const bool ac = lane < m && rs != 0;
        const unsigned long long fm = __ballot(fr), am = __ballot(ac);
        const int nF = __popcll(fm), nR = __popcll(am);
        const int N = nF + nR, W1 = N + 1;
        const int pF = __popcll(fm & below), pR = nF + __popcll(am & below);
        if (lane < n) {
          cpos[lane] = fr ? pF : -1;
          xs[lane] = cs == 1 ? L[0] : (cs == 2 ? U[0] : 0.0);
        }
        for (int q = lane; q < N * W1; q += WAVE) kkt[q] = 0.0;
        __syncthreads();
        if (fr) {
          kkt[pF * W1 + pF] = Q[0];
          kkt[pF * W1 + N] = -G[0];
        }
        if (ac) {
          double rhs = rs == 1 ? RL[0] : RU[0];
          for (int p = a.P.row_ptr[lane]; p < a.P.row_ptr[lane + 1]; ++p) {
            const int j = a.P.col_idx[p];
            const double av = vs[p];
            const int e = cpos[j];
            if (e >= 0) {
              kkt[pR * W1 + e] = av;
              kkt[e * W1 + pR] = -av;
            } else {
              rhs -= av * xs[j];
            }
          }
          kkt[pR * W1 + N] = rhs;
        }
        __syncthreads();
        double amax = 0.0;
        for (int q = lane; q < N * W1; q += WAVE) amax = fmax(amax, fabs(kkt[q]));
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) amax = fmax(amax, __shfl_xor(amax, off, WAVE));
        const double piv_min = 1e-11 * (amax > 0.0 ? amax : 1.0);
        int pr = 0, myrow = -1;
        for (int kk = 0; kk < N && pr < N; ++kk) {
          double pv = (lane >= pr && lane < N) ? fabs(kkt[lane * W1 + kk]) : -1.0;
          int pi = lane;
#pragma unroll
          for (int off = 32; off > 0; off >>= 1) {
            const double ov = __shfl_xor(pv, off, WAVE);
            const int oi = __shfl_xor(pi, off, WAVE);
            if (ov > pv || (ov == pv && oi < pi)) {
              pv = ov;
              pi = oi;
            }
          }
          if (!(pv > piv_min)) continue;  // dependent column: its unknown stays 0
          if (pi != pr && lane <= N) {
            const double t0 = kkt[pr * W1 + lane];
            kkt[pr * W1 + lane] = kkt[pi * W1 + lane];
            kkt[pi * W1 + lane] = t0;
          }
          __syncthreads();
          const double piv = kkt[pr * W1 + kk];
          const double rk = lane <= N ? kkt[pr * W1 + lane] / piv : 0.0;
          __syncthreads();
          if (lane <= N) kkt[pr * W1 + lane] = rk;
          for (int rr = 0; rr < N; ++rr) {
            if (rr == pr) continue;
            const double f = kkt[rr * W1 + kk];
            if (f != 0.0 && lane <= N) kkt[rr * W1 + lane] -= f * rk;
          }
          if (lane == kk) myrow = pr;
          ++pr;
          __syncthreads();
        }
        const double usol = (lane < N && myrow >= 0) ? kkt[myrow * W1 + N] : 0.0;
        const double uf = __shfl(usol, fr ? pF : 0, WAVE);
        const double ur = __shfl(usol, ac ? pR : 0, WAVE);
        double XU = 0.0;
        if (lane < n) XU = fr ? uf : xs[lane];
        if (lane < m) YN[0] = ac ? ur : 0.0;
        // ---- 3. check the clipped point
        if (lane < n) XN[0] = clampd(XU, L[0], U[0]);
        __syncthreads();
        if (lane < n) xs[lane] = XN[0];
        if (lane < m) ys[lane] = YN[0];
        __syncthreads();
        RW.dots(xs, part_r, DOT);
        if (lane < m) AXN[0] = DOT[0];
        double v[10];
        kkt_local(v);
        v[6] = v[7] = v[8] = v[9] = 0.0;
        block_sum<10>(v, red);
        double ep, ed, eg;
        kkt_measures(v, ep, ed, eg);
        if (ep <= a.tol && ed <= a.tol && eg <= a.tol) return true;
        // ---- primal-dual active-set update from the unclipped solution
        const bool clipped = __ballot(lane < n && XU != XN[0]) != 0ull;
        double AXU = AXN[0];
        const double LAMU = LAM[0] + Q[0] * (XU - XN[0]);
        if (clipped) {
          __syncthreads();
          if (lane < n) xs[lane] = XU;
          __syncthreads();
          RW.dots(xs, part_r, DOT);
          AXU = DOT[0];
        }
        __syncthreads();
        if (lane < n) {
          if (L[0] == U[0]) cs = 1;
          else if (isfinite(L[0]) && LAMU + (L[0] - XU) > 0.0) cs = 1;
          else if (isfinite(U[0]) && -LAMU + (XU - U[0]) > 0.0) cs = 2;
          else cs = 0;
        }
        if (lane < m) {
          if (RL[0] == RU[0]) rs = 1;
          else if (isfinite(RL[0]) && YN[0] + (RL[0] - AXU) > 0.0) rs = 1;
          else if (isfinite(RU[0]) && -YN[0] + (AXU - RU[0]) > 0.0) rs = 2;
          else rs = 0;
        }
      }
      XN[0] = sx;
      YN[0] = sy;
      AXN[0] = sa;
      LAM[0] = sl;
      __syncthreads();
      return false;
    }
  };

  // warm start: the previous PH iteration's active set usually still holds
  if constexpr (POL) {
    if (a.polish && a.warm) {
#pragma unroll
      for (int b = 0; b < CPT; ++b) XN[b] = X[b];
#pragma unroll
      for (int b = 0; b < RPT; ++b) {
        YN[b] = Y[b];
        AXN[b] = AX[b];
      }
      bool ok = polish_run(1e-9, POLISH_ROUNDS);
      if (ok) {
        stat = PH_STATUS_OPTIMAL;
        how = 1;
#pragma unroll
        for (int b = 0; b < CPT; ++b) X[b] = XN[b];
#pragma unroll
        for (int b = 0; b < RPT; ++b) Y[b] = YN[b];
        maxit_eff = 0;
      } else {
        // restore ys <- Y for the iteration
        if (tid < m) ys[tid] = Y[0];
        __syncthreads();
      }
    }
  }

  for (it = 0; it < maxit_eff; ++it) {
    const double cb = 1.0 / (double)(k + 2);
    const double ca = (double)(k + 1) * cb;
    const bool check = (it % chk) == 0 || it == maxit - 1;
    double dxx = 0.0, dyy = 0.0;

    // ---- column phase: x+ = clip((x - tau(g - A^T y)) / (1 + tau q))
    CL.dots(ys, part_c, DOT);
#pragma unroll
    for (int b = 0; b < CPT; ++b) {
      int j = tid + b * T;
      if (j < n) {
        const double aty = DOT[b];
        double xn = clampd((X[b] - tau * (G[b] - aty)) * IQ[b], L[b], U[b]);
        double d = xn - X[b];
        dxx += d * d;
        XN[b] = xn;
        X[b] = ca * ((1.0 + gam) * xn - gam * X[b]) + cb * Z0X[b];
        xs[j] = xn;
      }
    }
    __syncthreads();
    // ---- row phase: y+ = prox(y - sig A(2x+ - x))
    RW.dots(xs, part_r, DOT);
#pragma unroll
    for (int b = 0; b < RPT; ++b) {
      int i = tid + b * T;
      if (i < m) {
        const double axn = DOT[b];
        double v = Y[b] - sig * (2.0 * axn - AX[b]);
        double yn = fmax(v + sig * RL[b], 0.0) + fmin(v + sig * RU[b], 0.0);
        double d = yn - Y[b];
        dyy += d * d;
        YN[b] = yn;
        AXN[b] = axn;
        Y[b] = ca * ((1.0 + gam) * yn - gam * Y[b]) + cb * Z0Y[b];
        AX[b] = ca * ((1.0 + gam) * axn - gam * AX[b]) + cb * AZ0[b];
      }
    }
    ++k;
    if (!check) {
#pragma unroll
      for (int b = 0; b < RPT; ++b) {
        int i = tid + b * T;
        if (i < m) ys[i] = Y[b];
      }
      __syncthreads();
      continue;
    }
    // ---- check: KKT of the trial point (x+, y+) in the unscaled space
    __syncthreads();  // every thread done reading xs in the row phase
#pragma unroll
    for (int b = 0; b < RPT; ++b) {
      int i = tid + b * T;
      if (i < m) ys[i] = YN[b];
    }
    __syncthreads();
    double v[10];
    kkt_local(v);
    double ddx = 0.0, ddy = 0.0;
#pragma unroll
    for (int b = 0; b < CPT; ++b) {
      int j = tid + b * T;
      if (j < n) {
        double e = XN[b] - Z0X[b];
        ddx += e * e;
      }
    }
#pragma unroll
    for (int b = 0; b < RPT; ++b) {
      int i = tid + b * T;
      if (i < m) {
        double e = YN[b] - Z0Y[b];
        ddy += e * e;
      }
    }
    v[6] = ddx;
    v[7] = ddy;
    v[8] = dxx;
    v[9] = dyy;
    block_sum<10>(v, red);
    double ep, ed, eg;
    kkt_measures(v, ep, ed, eg);
    const double r = sqrt(omega * v[8] + v[9] / omega);
    d_r = r;
    if (ep <= a.tol && ed <= a.tol && eg <= a.tol) {
      stat = PH_STATUS_OPTIMAL;
#pragma unroll
      for (int b = 0; b < CPT; ++b) X[b] = XN[b];
#pragma unroll
      for (int b = 0; b < RPT; ++b) Y[b] = YN[b];
      ++it;
      break;
    }
    if constexpr (POL) {
      // near the optimum: guess the active set from the trial point and
      // solve its KKT system; accepted only if the KKT check passes
      const double err = fmax(ep, fmax(ed, eg));
      if (a.polish && err <= POLISH_START) {
        bool ok = polish_run(fmin(sqrt(err), 1e-3), POLISH_ROUNDS);
        if (ok) {
          stat = PH_STATUS_OPTIMAL;
          how = 2;
#pragma unroll
          for (int b = 0; b < CPT; ++b) X[b] = XN[b];
#pragma unroll
          for (int b = 0; b < RPT; ++b) Y[b] = YN[b];
          ++it;
          break;
        }
      }
    }
    bool restart = false;
    if (r_restart < 0.0) {
      r_restart = r;
    } else {
      restart = (r <= 0.2 * r_restart) || (r <= 0.8 * r_restart && r > r_prev) ||
                (k >= 0.36 * (double)(it + 1));
    }
    r_prev = r;
    // safeguard: every 8192 steps, a primal weight that has drifted more than
    // 100x from the data-based weight is reset (seen stalling on farmer warm
    // starts at ~1e-8 relative KKT, in both directions)
    const bool reset = it > 0 && ((it + 1) % 8192) < chk &&
                       (omega > 1e2 * omega0 || omega < 1e-2 * omega0);
    if (reset) {
      omega = omega0;
      restart = true;
    } else if (restart) {
      // PDLP primal weight update, smoothing 0.5
      const double dx = sqrt(v[6]), dy = sqrt(v[7]);
      if (dx > 1e-12 && dy > 1e-12) omega = exp(0.5 * log(dy / dx) + 0.5 * log(omega));
    }
    if (restart) {
      set_steps();
#pragma unroll
      for (int b = 0; b < CPT; ++b) X[b] = Z0X[b] = XN[b];
#pragma unroll
      for (int b = 0; b < RPT; ++b) {
        Y[b] = Z0Y[b] = YN[b];
        AX[b] = AZ0[b] = AXN[b];
      }
      k = 0;
      r_restart = r;
    }
    __syncthreads();  // all reads of ys (check col phase) done
#pragma unroll
    for (int b = 0; b < RPT; ++b) {
      int i = tid + b * T;
      if (i < m) ys[i] = Y[b];
    }
    __syncthreads();
  }

  // ---- write back (unscaled, scenario-fastest)
#pragma unroll
  for (int b = 0; b < CPT; ++b) {
    int j = tid + b * T;
    if (j < n) a.x[(size_t)j * S + s] = X[b] * DC[b];
  }
#pragma unroll
  for (int b = 0; b < RPT; ++b) {
    int i = tid + b * T;
    if (i < m) a.y[(size_t)i * S + s] = Y[b] * DR[b];
  }
  if (tid == 0) {
    a.omega[s] = omega;
    a.status[s] = stat;
    a.iters[s] = it;
    a.pobj[s] = out_pobj;
    a.dbound[s] = out_dobj;
    a.diag[PH_DIAG_W * s + 0] = d_ep;
    a.diag[PH_DIAG_W * s + 1] = d_ed;
    a.diag[PH_DIAG_W * s + 2] = d_eg;
    a.diag[PH_DIAG_W * s + 3] = d_r;
    a.diag[PH_DIAG_W * s + 4] = (double)how;
    if (stat != PH_STATUS_OPTIMAL) atomicAdd(&a.summary[0], 1ull);
    atomicAdd(&a.summary[1], (unsigned long long)it);
    atomicMax(&a.summary[2], (unsigned long long)it);
    if (how) atomicAdd(&a.summary[3], 1ull);
  }
}

// ------------------------------------------------------------------------
// nonanticipativity kernels (scenario-fastest, coalesced)
// ------------------------------------------------------------------------
__global__ void __launch_bounds__(256) xbar_accum_kernel(
    int S, const double *__restrict__ x, const double *__restrict__ pc,
    const int32_t *__restrict__ nonant_col, const int32_t *__restrict__ slot_k,
    const int32_t *__restrict__ s0, const int32_t *__restrict__ s1, int G,
    double *__restrict__ out) {
  __shared__ double red[MAX_WAVES * 2];
  const int g = blockIdx.x;
  const int k = slot_k[g];
  const double *xr = x + (size_t)nonant_col[k] * S;
  const double *pr = pc + (size_t)k * S;
  double v[2] = {0.0, 0.0};
  for (int s = s0[g] + threadIdx.x; s < s1[g]; s += blockDim.x) {
    double xv = xr[s], p = pr[s];
    v[0] += p * xv;
    v[1] += p * xv * xv;
  }
  block_sum<2>(v, red);
  if (threadIdx.x == 0) {
    out[g] = v[0];
    out[G + g] = v[1];
  }
}

__global__ void __launch_bounds__(256) update_w_kernel(
    int S, int K, const double *__restrict__ x, const int32_t *__restrict__ nonant_col,
    const double *__restrict__ sums, int G, const int32_t *__restrict__ gid,
    const double *__restrict__ rho, const double *__restrict__ wc,
    double *__restrict__ xbar, double *__restrict__ xsqbar, double *__restrict__ W,
    double *__restrict__ absdiff) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= S) return;
  double acc = 0.0;
  for (int k = 0; k < K; ++k) {
    const size_t o = (size_t)k * S + s;
    const int g = gid[o];
    const double xb = sums[g], xsq = sums[G + g];
    const double xv = x[(size_t)nonant_col[k] * S + s];
    xbar[o] = xb;
    xsqbar[o] = xsq;
    const double d = xv - xb;
    if (W) {
      double w = W[o] + rho[o] * d;
      if (wc) w *= wc[o];
      W[o] = w;
    }
    acc += fabs(d);
  }
  absdiff[s] = acc;
}

__global__ void __launch_bounds__(256) segment_sum_kernel(
    const double *__restrict__ v, const double *__restrict__ w,
    const int32_t *__restrict__ seg, double *__restrict__ out) {
  __shared__ double red[MAX_WAVES];
  const int r = blockIdx.x;
  double acc[1] = {0.0};
  for (int s = seg[r] + threadIdx.x; s < seg[r + 1]; s += blockDim.x)
    acc[0] += w ? w[s] * v[s] : v[s];
  block_sum<1>(acc, red);
  if (threadIdx.x == 0) out[r] = acc[0];
}

__global__ void __launch_bounds__(256) eval_obj_kernel(
    int S, int n, const double *__restrict__ c, const int32_t *__restrict__ slot_of_col,
    const double *__restrict__ x, const double *__restrict__ W,
    const double *__restrict__ rho, const double *__restrict__ xbar, double w_on,
    double prox_on, double *__restrict__ obj) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= S) return;
  double acc = 0.0;
  for (int j = 0; j < n; ++j) {
    const double xv = x[(size_t)j * S + s];
    acc += c[(size_t)j * S + s] * xv;
    const int k = slot_of_col[j];
    if (k >= 0) {
      const size_t o = (size_t)k * S + s;
      const double xb = xbar[o], r = rho[o];
      acc += w_on * W[o] * xv + prox_on * 0.5 * r * (xv * xv - 2.0 * xb * xv + xb * xb);
    }
  }
  obj[s] = acc;
}

}  // namespace

// --------------------------------------------------------------------------
// handle
// --------------------------------------------------------------------------
struct ph_batch {
  int S = 0, n = 0, m = 0, nnz = 0, K = 0;
  hipStream_t stream = nullptr;
  int32_t *d_row_ptr = nullptr, *d_col_idx = nullptr, *d_col_ptr = nullptr;
  int32_t *d_csc_row = nullptr, *d_csc_k = nullptr;
  int32_t *d_slot_of_col = nullptr, *d_nonant_col = nullptr;
  double *d_vals_s = nullptr, *d_dr = nullptr, *d_dc = nullptr, *d_eta = nullptr;
  double *d_c = nullptr, *d_l = nullptr, *d_u = nullptr, *d_rl = nullptr, *d_ru = nullptr;
  double *d_diag = nullptr;
  unsigned long long *d_summary = nullptr;
  // extra chunks of lines longer than LINE_D (see LineRegs)
  int xr = 0, xc = 0;
  int32_t *d_r_pb = nullptr, *d_r_pos = nullptr, *d_r_len = nullptr;
  int32_t *d_c_pb = nullptr, *d_c_pos = nullptr, *d_c_len = nullptr;
  bool bound = false;
  int per = 1, block = 64, ext = 0;
};

namespace {

template <typename T>
int dalloc(T **p, size_t count) {
  if (count == 0) count = 1;
  HIP_OK(hipMalloc((void **)p, count * sizeof(T)));
  return 0;
}

// Block size, lines (columns and rows) owned per thread and extra-chunk
// slots per thread.  Per-thread register state is ~30 VGPRs per owned
// column or row and 12 per extra chunk slot, so slots per thread stay <= 6
// (VGPR budget at two waves per SIMD); larger scenarios need the streaming
// kernel (not built).
bool pick_geometry(int n, int m, int xr, int xc, int *block, int *per, int *ext) {
  static const int G[][2] = {{64, 1},  {128, 1}, {256, 1}, {256, 2},
                             {512, 2}, {512, 3}, {512, 4}, {512, 6}};
  const int mx = n > m ? n : m;
  const int xx = xr > xc ? xr : xc;
  for (const auto &g : G) {
    if (mx > g[0] * g[1]) continue;
    int e = (xx + g[0] - 1) / g[0];
    if (e > 4) continue;
    *block = g[0];
    *per = g[1];
    *ext = e == 3 ? 4 : e;
    return true;
  }
  return false;
}

#define DISPATCH_EXT(BLK, PER, EXT, ...)                                              \
  do {                                                                               \
    if (EXT == 0) { constexpr int B_ = BLK, P_ = PER, E_ = 0; (void)E_; __VA_ARGS__; }          \
    else if (EXT == 1) { constexpr int B_ = BLK, P_ = PER, E_ = 1; (void)E_; __VA_ARGS__; }     \
    else if (EXT == 2) { constexpr int B_ = BLK, P_ = PER, E_ = 2; (void)E_; __VA_ARGS__; }     \
    else { constexpr int B_ = BLK, P_ = PER, E_ = 4; (void)E_; __VA_ARGS__; }                   \
  } while (0)

#define DISPATCH_GEOM(BLK, PER, EXT, ...)                                              \
  do {                                                                                \
    if (BLK == 64 && PER == 1) DISPATCH_EXT(64, 1, EXT, __VA_ARGS__);                 \
    else if (BLK == 128 && PER == 1) DISPATCH_EXT(128, 1, EXT, __VA_ARGS__);          \
    else if (BLK == 256 && PER == 1) DISPATCH_EXT(256, 1, EXT, __VA_ARGS__);          \
    else if (BLK == 256 && PER == 2) DISPATCH_EXT(256, 2, EXT, __VA_ARGS__);          \
    else if (BLK == 512 && PER == 2) DISPATCH_EXT(512, 2, EXT, __VA_ARGS__);          \
    else if (BLK == 512 && PER == 3) DISPATCH_EXT(512, 3, EXT, __VA_ARGS__);          \
    else if (BLK == 512 && PER == 4) DISPATCH_EXT(512, 4, EXT, __VA_ARGS__);          \
    else if (BLK == 512 && PER == 6) DISPATCH_EXT(512, 6, EXT, __VA_ARGS__);          \
    else return fail(PH_EINVAL, "internal: no kernel instance for this geometry");    \
  } while (0)

// Cut every line (row of the CSR view or column of the CSC view) into its
// owner's first LINE_D entries plus extra chunks of LINE_D.
void build_chunks(int lines, const std::vector<int32_t> &ptr, std::vector<int32_t> &pb,
                  std::vector<int32_t> &pos, std::vector<int32_t> &len) {
  pb.assign(lines + 1, 0);
  pos.clear();
  len.clear();
  for (int i = 0; i < lines; ++i) {
    pb[i] = (int32_t)pos.size();
    for (int p = ptr[i] + LINE_D; p < ptr[i + 1]; p += LINE_D) {
      pos.push_back(p);
      len.push_back(std::min(LINE_D, ptr[i + 1] - p));
    }
  }
  pb[lines] = (int32_t)pos.size();
}

}  // namespace

extern "C" {

const char *ph_version(void) { return PHGPU_VERSION; }

const char *ph_last_error(void) { return g_err.c_str(); }

int ph_batch_create(ph_batch_t *out, int32_t S, int32_t n, int32_t m, int32_t nnz,
                    const int32_t *row_ptr, const int32_t *col_idx, void *stream) {
  if (!out || S <= 0 || n <= 0 || m < 0 || nnz < 0 || !row_ptr || (nnz > 0 && !col_idx))
    return fail(PH_EINVAL, "ph_batch_create: bad arguments");
  if (row_ptr[0] != 0 || row_ptr[m] != nnz) return fail(PH_EINVAL, "ph_batch_create: row_ptr inconsistent with nnz");
  for (int i = 0; i < m; ++i)
    if (row_ptr[i + 1] < row_ptr[i]) return fail(PH_EINVAL, "ph_batch_create: row_ptr not monotone");
  for (int p = 0; p < nnz; ++p)
    if (col_idx[p] < 0 || col_idx[p] >= n) return fail(PH_EINVAL, "ph_batch_create: col_idx out of range");
  // CSC view of the shared pattern
  std::vector<int32_t> col_ptr(n + 1, 0), csc_row(nnz), csc_k(nnz);
  for (int p = 0; p < nnz; ++p) col_ptr[col_idx[p] + 1]++;
  for (int j = 0; j < n; ++j) col_ptr[j + 1] += col_ptr[j];
  std::vector<int32_t> fill(col_ptr.begin(), col_ptr.end() - 1);
  for (int i = 0; i < m; ++i)
    for (int p = row_ptr[i]; p < row_ptr[i + 1]; ++p) {
      int q = fill[col_idx[p]]++;
      csc_row[q] = i;
      csc_k[q] = p;
    }
  ph_batch *b = new ph_batch();
  b->S = S; b->n = n; b->m = m; b->nnz = nnz;
  b->stream = (hipStream_t)stream;
  std::vector<int32_t> rptr(row_ptr, row_ptr + m + 1);
  std::vector<int32_t> r_pb, r_pos, r_len, c_pb, c_pos, c_len;
  build_chunks(m, rptr, r_pb, r_pos, r_len);
  build_chunks(n, col_ptr, c_pb, c_pos, c_len);
  b->xr = (int)r_pos.size();
  b->xc = (int)c_pos.size();
  if (!pick_geometry(n, m, b->xr, b->xc, &b->block, &b->per, &b->ext)) {
    delete b;
    return fail(PH_EINVAL, "ph_batch_create: scenario has more than 3072 rows or columns (or too many "
                           "long rows/columns); the on-chip PDHG kernel does not cover it");
  }
  int rc = 0;
  if ((rc = dalloc(&b->d_row_ptr, m + 1)) || (rc = dalloc(&b->d_col_idx, nnz)) ||
      (rc = dalloc(&b->d_col_ptr, n + 1)) || (rc = dalloc(&b->d_csc_row, nnz)) ||
      (rc = dalloc(&b->d_csc_k, nnz)) || (rc = dalloc(&b->d_slot_of_col, n)) ||
      (rc = dalloc(&b->d_vals_s, (size_t)S * nnz)) || (rc = dalloc(&b->d_dr, (size_t)S * m)) ||
      (rc = dalloc(&b->d_dc, (size_t)S * n)) || (rc = dalloc(&b->d_eta, S)) ||
      (rc = dalloc(&b->d_c, (size_t)S * n)) || (rc = dalloc(&b->d_l, (size_t)S * n)) ||
      (rc = dalloc(&b->d_u, (size_t)S * n)) || (rc = dalloc(&b->d_rl, (size_t)S * m)) ||
      (rc = dalloc(&b->d_ru, (size_t)S * m)) || (rc = dalloc(&b->d_diag, (size_t)S * PH_DIAG_W)) ||
      (rc = dalloc(&b->d_summary, 4)) ||
      (rc = dalloc(&b->d_r_pb, m + 1)) || (rc = dalloc(&b->d_r_pos, b->xr)) ||
      (rc = dalloc(&b->d_r_len, b->xr)) || (rc = dalloc(&b->d_c_pb, n + 1)) ||
      (rc = dalloc(&b->d_c_pos, b->xc)) || (rc = dalloc(&b->d_c_len, b->xc))) {
    ph_batch_destroy(b);
    return rc;
  }
  std::vector<int32_t> noslot(n, -1);
  auto cp = [&](void *d, const void *h, size_t bytes) {
    return hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, b->stream);
  };
  if (cp(b->d_row_ptr, row_ptr, sizeof(int32_t) * (m + 1)) != hipSuccess ||
      (nnz && cp(b->d_col_idx, col_idx, sizeof(int32_t) * nnz) != hipSuccess) ||
      cp(b->d_col_ptr, col_ptr.data(), sizeof(int32_t) * (n + 1)) != hipSuccess ||
      (nnz && cp(b->d_csc_row, csc_row.data(), sizeof(int32_t) * nnz) != hipSuccess) ||
      (nnz && cp(b->d_csc_k, csc_k.data(), sizeof(int32_t) * nnz) != hipSuccess) ||
      cp(b->d_slot_of_col, noslot.data(), sizeof(int32_t) * n) != hipSuccess ||
      cp(b->d_r_pb, r_pb.data(), sizeof(int32_t) * (m + 1)) != hipSuccess ||
      cp(b->d_c_pb, c_pb.data(), sizeof(int32_t) * (n + 1)) != hipSuccess ||
      (b->xr && cp(b->d_r_pos, r_pos.data(), sizeof(int32_t) * b->xr) != hipSuccess) ||
      (b->xr && cp(b->d_r_len, r_len.data(), sizeof(int32_t) * b->xr) != hipSuccess) ||
      (b->xc && cp(b->d_c_pos, c_pos.data(), sizeof(int32_t) * b->xc) != hipSuccess) ||
      (b->xc && cp(b->d_c_len, c_len.data(), sizeof(int32_t) * b->xc) != hipSuccess) ||
      hipStreamSynchronize(b->stream) != hipSuccess) {
    ph_batch_destroy(b);
    return fail(PH_EHIP, "ph_batch_create: copying the pattern failed");
  }
  *out = b;
  return PH_OK;
}

int ph_batch_set_stream(ph_batch_t b, void *stream) {
  if (!b) return fail(PH_EINVAL, "null batch");
  b->stream = (hipStream_t)stream;
  return PH_OK;
}

static size_t scale_lds_bytes(const ph_batch *b) {
  return sizeof(double) * ((size_t)b->nnz + 2 * b->m + 2 * b->n + MAX_WAVES * 8);
}
static bool polish_fits(const ph_batch *b) {
  return b->block == WAVE && b->per == 1 && b->n + b->m <= POLISH_MAX;
}
static size_t solve_lds_bytes(const ph_batch *b) {
  size_t d = (size_t)b->n + b->m + b->xr + b->xc + MAX_WAVES * 10;
  size_t extra = 0;
  if (polish_fits(b)) {  // KKT matrix + free-column positions
    const size_t N = (size_t)b->n + b->m;
    extra = sizeof(double) * N * (N + 1) + sizeof(int32_t) * b->n;
  }
  return sizeof(double) * d + extra;
}

int ph_batch_bind(ph_batch_t b, const double *vals, const double *c, const double *l,
                  const double *u, const double *rl, const double *ru) {
  if (!b || (!vals && b->nnz) || !c || !l || !u || (b->m && (!rl || !ru)))
    return fail(PH_EINVAL, "ph_batch_bind: null argument");
  const size_t Sn = (size_t)b->S * b->n, Sm = (size_t)b->S * b->m;
  HIP_OK(hipMemcpyAsync(b->d_c, c, Sn * 8, hipMemcpyDeviceToDevice, b->stream));
  HIP_OK(hipMemcpyAsync(b->d_l, l, Sn * 8, hipMemcpyDeviceToDevice, b->stream));
  HIP_OK(hipMemcpyAsync(b->d_u, u, Sn * 8, hipMemcpyDeviceToDevice, b->stream));
  if (Sm) {
    HIP_OK(hipMemcpyAsync(b->d_rl, rl, Sm * 8, hipMemcpyDeviceToDevice, b->stream));
    HIP_OK(hipMemcpyAsync(b->d_ru, ru, Sm * 8, hipMemcpyDeviceToDevice, b->stream));
  }
  const size_t lds = scale_lds_bytes(b);
  if (lds > 160 * 1024) return fail(PH_EINVAL, "ph_batch_bind: scenario does not fit in LDS (nnz+2n+2m too large)");
  Pattern P{b->d_row_ptr, b->d_col_idx, b->d_col_ptr, b->d_csc_row, b->d_csc_k};
  DISPATCH_GEOM(b->block, b->per, 0, {
    hipLaunchKernelGGL((scale_kernel<B_, P_, P_>), dim3(b->S), dim3(B_), lds, b->stream,
                       b->S, b->n, b->m, b->nnz, P, vals, b->d_vals_s, b->d_dr, b->d_dc, b->d_eta);
  });
  HIP_OK(hipGetLastError());
  b->bound = true;
  return PH_OK;
}

int ph_batch_set_nonants(ph_batch_t b, int32_t K, const int32_t *nonant_col) {
  if (!b || K < 0 || (K && !nonant_col)) return fail(PH_EINVAL, "ph_batch_set_nonants: bad arguments");
  std::vector<int32_t> slot(b->n, -1);
  for (int k = 0; k < K; ++k) {
    if (nonant_col[k] < 0 || nonant_col[k] >= b->n) return fail(PH_EINVAL, "nonant column out of range");
    if (slot[nonant_col[k]] >= 0) return fail(PH_EINVAL, "nonant column listed twice");
    slot[nonant_col[k]] = k;
  }
  if (b->d_nonant_col) (void)hipFree(b->d_nonant_col);
  b->d_nonant_col = nullptr;
  int rc = dalloc(&b->d_nonant_col, K);
  if (rc) return rc;
  HIP_OK(hipMemcpyAsync(b->d_nonant_col, nonant_col, sizeof(int32_t) * (K ? K : 0), hipMemcpyHostToDevice, b->stream));
  HIP_OK(hipMemcpyAsync(b->d_slot_of_col, slot.data(), sizeof(int32_t) * b->n, hipMemcpyHostToDevice, b->stream));
  HIP_OK(hipStreamSynchronize(b->stream));
  b->K = K;
  return PH_OK;
}

int ph_pdhg_solve(ph_batch_t b, const double *W, const double *rho, const double *xbar,
                  double w_on, double prox_on, double *x, double *y, double *omega,
                  int32_t *status, int32_t *iters, double *pobj, double *dbound,
                  const ph_solve_opts *opts) {
  if (!b || !b->bound) return fail(PH_EINVAL, "ph_pdhg_solve: batch not bound");
  if (!x || (b->m && !y) || !omega || !status || !iters || !pobj || !dbound)
    return fail(PH_EINVAL, "ph_pdhg_solve: null output");
  if (b->K && (!W || !rho || !xbar)) return fail(PH_EINVAL, "ph_pdhg_solve: null W/rho/xbar");
  SolveArgs a;
  a.S = b->S; a.n = b->n; a.m = b->m; a.nnz = b->nnz;
  a.P = Pattern{b->d_row_ptr, b->d_col_idx, b->d_col_ptr, b->d_csc_row, b->d_csc_k};
  a.X = Chunks{b->xr, b->xc, b->d_r_pb, b->d_r_pos, b->d_r_len, b->d_c_pb, b->d_c_pos, b->d_c_len};
  a.vals_s = b->d_vals_s; a.dr = b->d_dr; a.dc = b->d_dc; a.eta = b->d_eta;
  a.c = b->d_c; a.l = b->d_l; a.u = b->d_u; a.rl = b->d_rl; a.ru = b->d_ru;
  a.slot_of_col = b->d_slot_of_col;
  a.W = W; a.rho = rho; a.xbar = xbar; a.w_on = w_on; a.prox_on = prox_on;
  a.x = x; a.y = y; a.omega = omega; a.status = status; a.iters = iters;
  a.pobj = pobj; a.dbound = dbound; a.diag = b->d_diag; a.summary = b->d_summary;
  a.tol = opts ? opts->tol : 1e-9;
  a.max_iters = opts ? opts->max_iters : 200000;
  a.check_every = opts ? opts->check_every : 64;
  a.warm = opts ? opts->warm_start : 1;
  a.refl = opts ? opts->reflection : 1.0;
  a.polish = (opts ? opts->polish : 1) && polish_fits(b);
  if (!(a.tol > 0.0) || a.max_iters <= 0) return fail(PH_EINVAL, "ph_pdhg_solve: bad options");
  const size_t lds = solve_lds_bytes(b);
  if (lds > 160 * 1024) return fail(PH_EINVAL, "ph_pdhg_solve: scenario does not fit in LDS");
  HIP_OK(hipMemsetAsync(b->d_summary, 0, 4 * sizeof(unsigned long long), b->stream));
  DISPATCH_GEOM(b->block, b->per, b->ext, {
    hipLaunchKernelGGL((pdhg_kernel<B_, P_, E_>), dim3(b->S), dim3(B_), lds, b->stream, a);
  });
  HIP_OK(hipGetLastError());
  return PH_OK;
}

int ph_xbar_accum(ph_batch_t b, const double *x, const double *prob_coeff, int32_t G,
                  const int32_t *slot_k, const int32_t *slot_s0, const int32_t *slot_s1,
                  double *out_sums) {
  if (!b || !x || !prob_coeff || G <= 0 || !slot_k || !slot_s0 || !slot_s1 || !out_sums)
    return fail(PH_EINVAL, "ph_xbar_accum: bad arguments");
  if (!b->d_nonant_col || b->K == 0) return fail(PH_EINVAL, "ph_xbar_accum: no nonants declared");
  hipLaunchKernelGGL(xbar_accum_kernel, dim3(G), dim3(256), 0, b->stream, b->S, x, prob_coeff,
                     b->d_nonant_col, slot_k, slot_s0, slot_s1, G, out_sums);
  HIP_OK(hipGetLastError());
  return PH_OK;
}

int ph_update_w(ph_batch_t b, const double *x, const double *sums, int32_t G, const int32_t *gid,
                const double *rho, const double *w_coeff, double *xbar, double *xsqbar, double *W,
                double *absdiff) {
  if (!b || !x || !sums || G <= 0 || !gid || !rho || !xbar || !xsqbar || !absdiff)
    return fail(PH_EINVAL, "ph_update_w: bad arguments");
  if (!b->d_nonant_col || b->K == 0) return fail(PH_EINVAL, "ph_update_w: no nonants declared");
  hipLaunchKernelGGL(update_w_kernel, dim3((b->S + 255) / 256), dim3(256), 0, b->stream, b->S,
                     b->K, x, b->d_nonant_col, sums, G, gid, rho, w_coeff, xbar, xsqbar, W, absdiff);
  HIP_OK(hipGetLastError());
  return PH_OK;
}

int ph_segment_sum(ph_batch_t b, const double *v, const double *w, int32_t R, const int32_t *seg,
                   double *out) {
  if (!b || !v || R <= 0 || !seg || !out) return fail(PH_EINVAL, "ph_segment_sum: bad arguments");
  hipLaunchKernelGGL(segment_sum_kernel, dim3(R), dim3(256), 0, b->stream, v, w, seg, out);
  HIP_OK(hipGetLastError());
  return PH_OK;
}

int ph_eval_objective(ph_batch_t b, const double *x, const double *W, const double *rho,
                      const double *xbar, double w_on, double prox_on, double *obj) {
  if (!b || !b->bound || !x || !obj) return fail(PH_EINVAL, "ph_eval_objective: bad arguments");
  if (b->K && (!W || !rho || !xbar)) return fail(PH_EINVAL, "ph_eval_objective: null W/rho/xbar");
  hipLaunchKernelGGL(eval_obj_kernel, dim3((b->S + 255) / 256), dim3(256), 0, b->stream, b->S,
                     b->n, b->d_c, b->d_slot_of_col, x, W, rho, xbar, w_on, prox_on, obj);
  HIP_OK(hipGetLastError());
  return PH_OK;
}

int ph_batch_get_diag(ph_batch_t b, double *out) {
  if (!b || !out) return fail(PH_EINVAL, "ph_batch_get_diag: bad arguments");
  HIP_OK(hipMemcpyAsync(out, b->d_diag, sizeof(double) * PH_DIAG_W * (size_t)b->S, hipMemcpyDeviceToHost, b->stream));
  HIP_OK(hipStreamSynchronize(b->stream));
  return PH_OK;
}

int ph_batch_solve_summary(ph_batch_t b, int64_t *out) {
  if (!b || !out) return fail(PH_EINVAL, "ph_batch_solve_summary: bad arguments");
  unsigned long long h[4];
  HIP_OK(hipMemcpyAsync(h, b->d_summary, sizeof(h), hipMemcpyDeviceToHost, b->stream));
  HIP_OK(hipStreamSynchronize(b->stream));
  for (int i = 0; i < 4; ++i) out[i] = (int64_t)h[i];
  return PH_OK;
}

int ph_batch_sync(ph_batch_t b) {
  if (!b) return fail(PH_EINVAL, "null batch");
  HIP_OK(hipStreamSynchronize(b->stream));
  return PH_OK;
}

void ph_batch_destroy(ph_batch_t b) {
  if (!b) return;
  void *ptrs[] = {b->d_row_ptr, b->d_col_idx, b->d_col_ptr, b->d_csc_row, b->d_csc_k,
                  b->d_slot_of_col, b->d_nonant_col, b->d_vals_s, b->d_dr, b->d_dc,
                  b->d_eta, b->d_c, b->d_l, b->d_u, b->d_rl, b->d_ru, b->d_diag, b->d_summary,
                  b->d_r_pb, b->d_r_pos, b->d_r_len, b->d_c_pb, b->d_c_pos, b->d_c_len};
  for (void *p : ptrs)
    if (p) (void)hipFree(p);
  delete b;
}

}  // extern "C"
