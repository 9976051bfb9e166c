// gp_fit.hip -- GP hyper-parameter fit on device: log-marginal likelihood and its
// gradient for a batch of hyper-parameter vectors (gfx950, fp64).
//
// SURVEY §8a G1 / §8f rank 1.  skopt's Optimizer.tell refits
//   C(1,(0.01,1000)) * Matern(ls, (0.01,100), nu=2.5) + WhiteKernel()
// with sklearn's GaussianProcessRegressor(normalize_y=True, alpha=1e-10):
// L-BFGS-B over theta = log[amp, ls_0..ls_{d-1}, noise] from the kernel's start
// and n_restarts_optimizer uniform draws, each evaluation being
// log_marginal_likelihood(theta, eval_gradient=True)
// (sklearn gaussian_process/_gpr.py:296-337 and :537-655, kernels.py:1596-1724).
// The reference reaches it from Coordinator.fit (/root/reference/coordinator.py:63-79).
//
// One workgroup (1024 threads) evaluates one theta; a launch covers a batch of
// thetas (the restarts advance in lockstep on the host), so the fit costs one
// launch per L-BFGS iteration instead of B host evaluations.
//
// Per workgroup, n <= 200 (the factor fits the 160 KB LDS as a packed triangle):
//   1. K = amp * Matern52(|x_i/ls - x_j/ls|) + (noise + 1e-10) I   -> LDS, packed
//      lower, column-major
//   2. Cholesky in LDS, blocked by 8-column panels (update / diagonal block /
//      rows below, three barriers per panel); the global variant is right-looking,
//      one barrier per column
//   3. the factor moves to the global workspace (row-major packed) and L^-1 is
//      built in the LDS (row-major packed), blocked by 64 rows: diagonal blocks
//      inverted in parallel, then block rows from the top
//   4. z = L^-1 y, alpha = L^-T z;  lml = -y.alpha/2 - sum log L_jj - n/2 log 2pi
//   5. per pair (i >= j): K^-1_ij = sum_m L^-1_mi L^-1_mj (LDS), W = a_i a_j - K^-1_ij,
//      recompute dK_ij/dtheta and accumulate W dK (x2 off the diagonal)
//   6. fixed-order reduction -> grad = 0.5 * sum_ij W_ij dK_ij/dtheta
// For n > 200 the same code runs with the factor and L^-1 in the global workspace.
// Everything is deterministic: fixed summation orders, no atomics.

#include "mpo_internal.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <string>
#include <vector>

namespace {

constexpr int kFitThreads = 1024;
constexpr int kFitWaves = kFitThreads / 64;
constexpr int kFitMaxN = 2048;
constexpr int kFitLdsMaxN = 200;  // 200*201/2 doubles = 160800 B of the 163840 B LDS
constexpr double kSqrt5 = 2.236067977499789696409173668731276235;
constexpr double kLog2Pi = 1.837877066409345483560659472811235280;
constexpr double kFitJitter = 1e-10;  // sklearn GaussianProcessRegressor alpha (_gpr.py:207)

struct LmlArgs {
    const double* X;      // [n][d]
    const double* y;      // [n] normalised targets
    int n, d;
    const double* theta;  // [B][d+2]
    double* lml;          // [B]
    double* grad;         // [B][d+2]
    int32_t* info;        // [B]
    double* ws;           // per theta: ws_stride doubles
    long long ws_stride;
    int stop;             // diagnostics only (env MPO_FIT_DEBUG): return after phase 1/2/3/4
    const double* theta_src;  // fused split sweep, host-staged call: theta in pinned host memory (device
                              // view), read by sw_xs_build_kernel and copied to `theta`; else nullptr
};

__host__ __device__ inline long long fit_tri(long long n) { return n * (n + 1) / 2; }

// per-theta workspace (doubles): xs [n][d] | z [n] | alpha [n] | factor, packed [n(n+1)/2]
// | L^-1 [n][n] (global variant only)
__host__ __device__ inline long long fit_ws_doubles(int n, int d, bool lds) {
    auto al = [](long long x) { return (x + 31) & ~31LL; };
    return al((long long)n * d) + 2 * al(n) + al(fit_tri(n)) + (lds ? 0 : al((long long)n * n));
}

__device__ __forceinline__ double wave_sum_bcast(double v) {
    // fixed butterfly; lane 0's result is broadcast so every lane holds the same bits
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
    return __shfl(v, 0);
}

// v_readlane of a double at a wave-uniform lane (two 32-bit halves -> SGPRs)
__device__ __forceinline__ double readlane_f64(double v, int l) {
    const unsigned long long u = __double_as_longlong(v);
    const unsigned lo = __builtin_amdgcn_readlane((unsigned)u, l);
    const unsigned hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), l);
    return __longlong_as_double(((unsigned long long)hi << 32) | lo);
}

template <bool kLds, int DP>
__global__ __launch_bounds__(kFitThreads) void lml_grad_kernel(LmlArgs a) {
    extern __shared__ __attribute__((aligned(16))) double fsm[];
    const int b = blockIdx.x;
    const int n = a.n, d = a.d;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const double* th = a.theta + (long long)b * (d + 2);
    auto al = [](long long x) { return (x + 31) & ~31LL; };
    double* ws = a.ws + (long long)b * a.ws_stride;
    double* xs = ws;
    double* z = xs + al((long long)n * d);
    double* alpha = z + al(n);
    double* Lg = alpha + al(n);              // global packed factor
    double* Linv_g = Lg + al(fit_tri(n));    // global variant: L^-1 [n][n]
    // LDS variant: the factor is built in LDS (column-major packed) and copied to Lg
    // (row-major packed) before L^-1 takes the LDS over (row-major packed).
    // Global variant: the factor lives in Lg column-major, L^-1 in Linv_g.
    double* Lp = kLds ? fsm : Lg;
    auto cidx = [n](int i, int j) { return j * n - j * (j - 1) / 2 + (i - j); };
    auto ridx = [](int i, int j) { return i * (i + 1) / 2 + j; };

    // kernel.theta setter: params = exp(theta) (sklearn kernels.py Hyperparameter theta)
    const double amp = exp(th[0]);
    const double noise = exp(th[d + 1]);
    double ls[DP];
#pragma unroll
    for (int c = 0; c < DP; ++c) ls[c] = c < d ? exp(th[1 + c]) : 1.0;

    // ---- 1. K (packed lower, column-major) from xs = X / ls (pdist(X / ls))
    for (int e = tid; e < n * d; e += kFitThreads) {
        const int c = e % d;
        double lc = 1.0;
#pragma unroll
        for (int q = 0; q < DP; ++q)
            if (q == c) lc = ls[q];
        xs[e] = a.X[e] / lc;
    }
    __syncthreads();
    for (int j = wave; j < n; j += kFitWaves) {
        double xj[DP];
#pragma unroll
        for (int c = 0; c < DP; ++c) xj[c] = c < d ? xs[j * d + c] : 0.0;
        for (int i = j + lane; i < n; i += 64) {
            double v;
            if (i == j) {
                v = amp * 1.0 + noise + kFitJitter;
            } else {
                double r2 = 0.0;
#pragma unroll
                for (int c = 0; c < DP; ++c)
                    if (c < d) {
                        const double t = xs[i * d + c] - xj[c];
                        r2 += t * t;
                    }
                const double k = sqrt(r2) * kSqrt5;
                v = amp * ((1.0 + k + k * k / 3.0) * exp(-k));
            }
            Lp[cidx(i, j)] = v;
        }
    }
    __syncthreads();
    if (a.stop == 1) return;

    // ---- 2. Cholesky
    double logdet = 0.0, prev_rs = 0.0;
    int fail = 0;
    if (kLds) {
        // Blocked by PW-column panels, three barriers per panel instead of one per column:
        //  (u) A[p0:, panel] -= L[p0:, :p0] L[panel, :p0]^T   (all waves; task = column j
        //      x 64-row chunk, lane = row: column-major reads are lane-contiguous)
        //  (d) the diagonal block by wave 0, left-looking (lane = row; L_jj comes from
        //      lane j with readlane, so the wave needs no barrier between columns)
        //  (s) the rows below the block, left-looking against the finished block
        // A non-positive / non-finite pivot propagates (sqrt -> NaN or 0) and is found
        // by the diagonal scan below.
        constexpr int PW = 8;   // panel width (a multiple of 8: the update's k batches)
        for (int p0 = 0; p0 < n; p0 += PW) {
            const int pe = min(p0 + PW, n);
            if (p0 > 0) {
                const int nch = (n - p0 + 63) >> 6;
                for (int t = wave; t < (pe - p0) * nch; t += kFitWaves) {
                    const int j = p0 + t / nch, i = p0 + 64 * (t % nch) + lane;
                    const bool act = i >= j && i < n;
                    const int ir = act ? i : j;
                    double s0 = 0.0, s1 = 0.0;
                    // cidx(r, k+1) - cidx(r, k) = n - k - 1 for every row r, so one running
                    // address serves both rows (L_jk sits ir - j doubles before L_{ir,k})
                    const int dlt = ir - j;
                    int ad = ir;  // cidx(ir, 0)
                    for (int k = 0; k < p0; k += 8) {
                        double x[8], y[8];
#pragma unroll
                        for (int u = 0; u < 8; ++u) {
                            x[u] = fsm[ad];
                            y[u] = fsm[ad - dlt];
                            ad += n - (k + u) - 1;
                        }
#pragma unroll
                        for (int u = 0; u < 8; ++u) {
                            if (u & 1) s1 += x[u] * y[u];
                            else s0 += x[u] * y[u];
                        }
                    }
                    if (act) fsm[cidx(i, j)] -= s0 + s1;
                }
                __syncthreads();
            }
            // left-looking panel dot: sum_{k=p0}^{j-1} L_rk L_jk for row r >= j (j - p0 < PW):
            // all loads issued at once at clamped (valid) addresses, summed in k order
            auto pdot = [&](int r, int j) -> double {
                double x[PW - 1], y[PW - 1];
#pragma unroll
                for (int u = 0; u < PW - 1; ++u) {
                    const int k = min(p0 + u, j);
                    x[u] = fsm[cidx(r, k)];
                    y[u] = fsm[cidx(j, k)];
                }
                double s = 0.0;
#pragma unroll
                for (int u = 0; u < PW - 1; ++u)
                    if (p0 + u < j) s += x[u] * y[u];
                return s;
            };
            if (wave == 0) {
                const int i = p0 + lane;
                const bool act = i < pe;
                for (int j = p0; j < pe; ++j) {
                    const int ir = (act && i >= j) ? i : j;
                    const double s = fsm[cidx(ir, j)] - pdot(ir, j);
                    const double ljj = sqrt(readlane_f64(s, j - p0));
                    if (act && i >= j) fsm[cidx(i, j)] = i == j ? ljj : s / ljj;
                }
            }
            __syncthreads();
            if (pe < n) {
                for (int c = wave; 64 * c < n - pe; c += kFitWaves) {
                    const int i = pe + 64 * c + lane;
                    const bool act = i < n;
                    const int ir = act ? i : n - 1;
                    for (int j = p0; j < pe; ++j) {
                        const double s = fsm[cidx(ir, j)] - pdot(ir, j);
                        if (act) fsm[cidx(i, j)] = s / fsm[cidx(j, j)];
                    }
                }
                __syncthreads();
            }
        }
        // every wave scans the diagonal the same way (same bits): first bad pivot, log det
        int f = 0;
        double ld = 0.0;
        for (int j = lane; j < n; j += 64) {
            const double r = fsm[cidx(j, j)];
            if (!(r > 0.0) || !isfinite(r)) {
                if (!f) f = j + 1;
            } else {
                ld += log(r);
            }
        }
        int fm = f ? f : 0x7fffffff;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) fm = min(fm, __shfl_xor(fm, off));
        fail = fm == 0x7fffffff ? 0 : fm;
        logdet = wave_sum_bcast(ld);
    }
    for (int j = 0; j < (kLds ? 0 : n); ++j) {
        const double dj = Lp[cidx(j, j)];
        if (!(dj > 0.0) || !isfinite(dj)) { fail = j + 1; break; }  // uniform: every thread reads dj
        const double rs = sqrt(dj);
        logdet += log(rs);
        const double inv = 1.0 / dj;
        if (j > 0) {  // finalise column j-1 (not read by this step's update)
            const int c0 = cidx(j - 1, j - 1);
            for (int e = tid; e < n - j + 1; e += kFitThreads) Lp[c0 + e] = e == 0 ? prev_rs : Lp[c0 + e] / prev_rs;
        }
        const int cj = cidx(j, j);
        for (int k = j + 1 + wave; k < n; k += kFitWaves) {
            const double lkj = Lp[cj + (k - j)] * inv;
            const int ck = cidx(k, k);
            for (int i = k + lane; i < n; i += 64) Lp[ck + (i - k)] -= Lp[cj + (i - j)] * lkj;
        }
        prev_rs = rs;
        __syncthreads();
    }
    if (fail) {  // sklearn: LinAlgError -> (-inf, zeros)
        if (tid == 0) { a.lml[b] = -INFINITY; a.info[b] = fail; }
        for (int c = tid; c < d + 2; c += kFitThreads) a.grad[(long long)b * (d + 2) + c] = 0.0;
        return;
    }
    if (!kLds && tid == 0) Lp[cidx(n - 1, n - 1)] = prev_rs;
    __syncthreads();
    if (a.stop == 2) return;

    // ---- 3. L^-1 by columns: thread c forward-substitutes e_c.  Row i of L is read
    // wave-uniformly (scalar loads); the solution column is the thread's own
    // (LDS in the LDS variant).  Entries above the diagonal are never stored or read.
    if (kLds) {
        for (int i = wave; i < n; i += kFitWaves)
            for (int j = lane; j <= i; j += 64) Lg[ridx(i, j)] = fsm[cidx(i, j)];
        __syncthreads();
    }
    auto lrow = [&](int i, int k) -> double { return kLds ? Lg[ridx(i, k)] : Lg[cidx(i, k)]; };
    auto lv = [&](int m, int j) -> double { return kLds ? fsm[ridx(m, j)] : Linv_g[m * n + j]; };
    auto lv_set = [&](int m, int j, double v) {
        if (kLds) fsm[ridx(m, j)] = v;
        else Linv_g[m * n + j] = v;
    };
    if (kLds) {
        // Blocked in 64-row blocks (n <= 200: at most 4), the dtrtri scheme:
        //  3a. every diagonal block is inverted at once, one wave per block, thread c
        //      forward-substituting e_c inside its block (chains of <= 64 rows
        //      instead of n);
        //  3b. block row bi, from the top: T = L[bi][:bi] X[:bi][bj] (all 16 waves,
        //      T written where X[bi][bj] goes), then X[bi][bj] = -inv(L[bi][bi]) T in
        //      place (each wave owns whole columns, so its reads of T precede its
        //      writes).
        const int nblk = (n + 63) >> 6;
        if (wave < nblk) {
            // row i of the block's L is held across the wave (lane l: L_{i,c0+l}) and
            // read with readlane (k is wave-uniform); row i+1 loads while i is used
            const int c0 = wave * 64, ce = min(c0 + 64, n);
            const int c = c0 + lane;
            const int cr = c < ce ? c : ce - 1;  // lanes past the block read a valid column, store nothing
            auto ld = [&](int i) -> double { return (i < ce && c <= i) ? Lg[ridx(i, c)] : 0.0; };
            double cur = ld(c0);
            for (int i = c0; i < ce; ++i) {
                const double nxt = ld(i + 1);
                double s0 = 0.0, s1 = 0.0;
                int k = c0;
                // batches of 8: all LDS loads issued before the FMAs
                for (; k + 7 < i; k += 8) {
                    double v[8];
                    int r = ridx(k, cr);
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        v[u] = fsm[r];
                        r += k + u + 1;
                    }
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        const double l = readlane_f64(cur, k + u - c0);
                        if (u & 1) s1 += k + u >= cr ? l * v[u] : 0.0;
                        else s0 += k + u >= cr ? l * v[u] : 0.0;
                    }
                }
                for (; k < i; ++k) s0 += k >= cr ? readlane_f64(cur, k - c0) * fsm[ridx(k, cr)] : 0.0;
                const double lii = readlane_f64(cur, i - c0);
                const double x = i == cr ? 1.0 / lii : -(s0 + s1) / lii;
                if (c < ce && i >= c) fsm[ridx(i, c)] = x;
                cur = nxt;
            }
        }
        __syncthreads();
        for (int bi = 1; bi < nblk; ++bi) {
            const int bi0 = bi * 64, bie = min(bi0 + 64, n), rows = bie - bi0;
            // T_ic = sum_{k=c}^{bi0-1} L_ik X_kc: wave task (row i, column block bj),
            // lane = column; L_i,k for k < bi0 held in registers (chunk q: k = 64q + lane)
            for (int t = wave; t < rows * bi; t += kFitWaves) {
                const int i = bi0 + t / bi, bj = t % bi;
                const int c = bj * 64 + lane;
                double lr[3];
#pragma unroll
                for (int q = 0; q < 3; ++q) lr[q] = (q >= bj && q < bi) ? Lg[ridx(i, 64 * q + lane)] : 0.0;
                double s0 = 0.0, s1 = 0.0;
#pragma unroll
                for (int q = 0; q < 3; ++q) {
                    if (q < bj || q >= bi) continue;
                    for (int kk = 0; kk < 64; kk += 8) {
                        const int k = 64 * q + kk;
                        double v[8];
                        int r = ridx(k, c);
#pragma unroll
                        for (int u = 0; u < 8; ++u) {
                            v[u] = fsm[r];
                            r += k + u + 1;
                        }
#pragma unroll
                        for (int u = 0; u < 8; ++u) {
                            const double l = readlane_f64(lr[q], kk + u);
                            if (u & 1) s1 += k + u >= c ? l * v[u] : 0.0;
                            else s0 += k + u >= c ? l * v[u] : 0.0;
                        }
                    }
                }
                fsm[ridx(i, c)] = s0 + s1;
            }
            __syncthreads();
            // X_ic = -sum_{m=bi0}^{i} inv(L_bb)_im T_mc: lane = row, wave-owned columns
            // c = wave + 16 j (64 bi columns); T_mc is a broadcast LDS read
            {
                const int i = bi0 + lane;
                const int ir = i < bie ? i : bie - 1;
                const int ncol = 4 * bi;  // 64 bi / 16 waves
                double acc[12];
#pragma unroll
                for (int j = 0; j < 12; ++j) acc[j] = 0.0;
                for (int m = bi0; m < bie; ++m) {
                    const double dm = m <= ir ? fsm[ridx(ir, m)] : 0.0;
                    const int rm = ridx(m, 0);
#pragma unroll
                    for (int j = 0; j < 12; ++j)
                        if (j < ncol) acc[j] += dm * fsm[rm + wave + 16 * j];
                }
#pragma unroll
                for (int j = 0; j < 12; ++j)
                    if (j < ncol && i < bie) fsm[ridx(i, wave + 16 * j)] = -acc[j];
            }
            __syncthreads();
        }
    } else {
        for (int c0 = wave * 64; c0 < n; c0 += kFitThreads) {
            const int c = c0 + lane;
            const int cr = c < n ? c : n - 1;
            for (int i = c0; i < n; ++i) {
                double s0 = 0.0;
                for (int k = c0; k < i; ++k) s0 += k >= cr ? lrow(i, k) * lv(k, cr) : 0.0;
                const double lii = lrow(i, i);
                const double x = i == cr ? 1.0 / lii : -s0 / lii;
                if (c < n && i >= c) lv_set(i, c, x);
            }
        }
    }
    __syncthreads();
    if (a.stop == 3) return;

    // ---- 4. alpha = L^-T L^-1 y
    for (int i = tid; i < n; i += kFitThreads) {
        double s = 0.0;
        for (int k = 0; k <= i; ++k) s += lv(i, k) * a.y[k];
        z[i] = s;
    }
    __syncthreads();
    for (int j = tid; j < n; j += kFitThreads) {
        double s = 0.0;
        for (int i = j; i < n; ++i) s += lv(i, j) * z[i];
        alpha[j] = s;
    }
    __syncthreads();
    if (a.stop == 4) return;

    // ---- 5. pairs (i >= j): W_ij dK_ij / dtheta
    double g[DP + 2];
#pragma unroll
    for (int c = 0; c < DP + 2; ++c) g[c] = 0.0;
    for (int i = wave; i < n; i += kFitWaves) {
        const double ai = alpha[i];
        double xi[DP];
#pragma unroll
        for (int c = 0; c < DP; ++c) xi[c] = c < d ? xs[i * d + c] : 0.0;
        for (int j = lane; j <= i; j += 64) {
            double k0 = 0.0, k1 = 0.0;
            int m = i;
            if (kLds) {
                int r = ridx(i, 0);  // start of row m (packed row-major), advanced by m + 1
                // batches of 8 rows: all 16 LDS loads issued before the FMAs
                for (; m + 7 < n; m += 8) {
                    double x[8], y[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        x[u] = fsm[r + i];
                        y[u] = fsm[r + j];
                        r += m + u + 1;
                    }
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        if (u & 1) k1 += x[u] * y[u];
                        else k0 += x[u] * y[u];
                    }
                }
                for (; m < n; ++m) {
                    k0 += fsm[r + i] * fsm[r + j];
                    r += m + 1;
                }
            } else {
                for (; m < n; ++m) k0 += lv(m, i) * lv(m, j);
            }
            const double kinv = k0 + k1;
            const double W = (ai * alpha[j] - kinv) * (i == j ? 1.0 : 2.0);
            // Matern gradient (kernels.py:1747-1767): D = (x_i - x_j)^2 / ls^2
            double D[DP], r2 = 0.0;
#pragma unroll
            for (int c = 0; c < DP; ++c) {
                if (c < d) {
                    // (x_i/ls - x_j/ls)^2: xs is phase 1's X / ls (no division per pair)
                    const double t = xi[c] - xs[j * d + c];
                    D[c] = t * t;
                    r2 += D[c];
                } else {
                    D[c] = 0.0;
                }
            }
            const double s = sqrt(5.0 * r2);
            const double e = exp(-s);
            const double Mij = i == j ? 1.0 : (1.0 + s + s * s / 3.0) * e;
            g[0] += W * (amp * Mij);
            const double f = W * amp * (5.0 / 3.0) * (s + 1.0) * e;
#pragma unroll
            for (int c = 0; c < DP; ++c) g[1 + c] += f * D[c];
            if (i == j) g[DP + 1] += W * noise;
        }
    }

    // ---- 6. fixed-order reduction: lanes (butterfly) -> waves (LDS, in order)
    __syncthreads();  // the pair pass is done with the LDS copy of L^-1
    double* red = fsm;  // [kFitWaves][DP + 2]
#pragma unroll
    for (int c = 0; c < DP + 2; ++c) {
        const double v = wave_sum_bcast(g[c]);
        if (lane == 0) red[wave * (DP + 2) + c] = v;
    }
    __syncthreads();
    if (tid == 0) {
        double ya = 0.0;
        for (int i = 0; i < n; ++i) ya += a.y[i] * alpha[i];
        a.lml[b] = -0.5 * ya - logdet - 0.5 * n * kLog2Pi;
        a.info[b] = 0;
        double* out = a.grad + (long long)b * (d + 2);
        for (int c = 0; c < d + 2; ++c) {
            const int src = c == 0 ? 0 : (c == d + 1 ? DP + 1 : c);
            double s = 0.0;
            for (int w = 0; w < kFitWaves; ++w) s += red[w * (DP + 2) + src];
            out[c] = 0.5 * s;
        }
    }
}

// ===========================================================================
// Block sweep (n > kSplitMinN): K^-1 and log det K by the symmetric sweep operator
// over 32-wide pivot blocks, trailing updates on v_mfma_f64_16x16x4.
//
// Sweeping pivot block k of a symmetric A (Goodnight's sweep, block form):
//     A_kk <- -A_kk^-1,   A_ik <- A_ik A_kk^-1,   A_ij <- A_ij - A_ik A_kk^-1 A_kj
// for i, j != k; after every block is swept A = -K^-1, and log det K is the sum of
// the log determinants of the pivot blocks at their sweep (the Schur complements
// a Cholesky factorisation meets).  Work: n^3 flops, all in rank-32 MFMA updates
// of the lower triangle; no L^-1, and the pair phase reads K^-1 directly instead
// of forming L^-T L^-1 entry by entry.  Padding rows/columns n..np carry the
// identity, so they never couple to K.
//
// Spread over the device: sw_xs_build_kernel (xs, K; many workgroups), one
// sw_step_kernel per pivot block (every workgroup sweeps the 32x32 pivot block
// in its wave 0 -- a non-positive pivot is sklearn's Cholesky LinAlgError --
// then each wave updates one lower 16x16 tile A_IJ -= G_I C_J^T, G_I = C_I P^-1),
// sw_alpha_kernel, sw_pairs_final_kernel (gradient pairs, last workgroup sums the
// partials and writes the LML).  (A single-workgroup form of the same sweep ran
// every trailing update on one CU: 2.45 ms per launch at n = 500 vs 0.86 ms.)
constexpr int kSwNb = 32;

typedef double f64x4 __attribute__((ext_vector_type(4)));

__host__ __device__ inline long long sw_np(int n) { return (n + kSwNb - 1) / kSwNb * kSwNb; }

constexpr int kSplitMinN = 48;    // past it the split beats both single-workgroup kernels (0.09 vs 0.20 ms at n = 64)
constexpr int kStepWaves = 4;   // waves per sw_step workgroup; all of them share the pivot sweep
constexpr int kUpdTilesPerWave = 1;   // one lower tile per wave: latency-bound steps want many waves
// sw_step workgroups per launch before waves take more tiles (one per CU).  Chains at
// n = 448, 8 / 16 threads: 72 / 82 refits/s with one tile per wave, 93 / 120 at 256,
// 98 / 112 at 512, 84 / 94 at 1024, 79 / 96 at 128, 68 / 85 at 64; n = 256: 150 / 189
// -> 175 / 210 (profiles/r05/tpw_*.log); MPO_FIT_STEP_WG overrides it for sweeps
constexpr long long kStepWgTarget = 256;

// per-theta workspace (doubles): xs | alpha | A [np][np] | C0, C1 [np][32]
// | P^-1 [32][32] | logdet, fail.  C_k (block column k before sweep k, row-major
// [np][32]) lives in C[k & 1]: the update kernel of step k writes C_{k+1} as it
// produces those entries, so the pivot kernel never re-reads a block column of A.
__host__ __device__ inline long long ss_ws_doubles(int n, int d) {
    auto al = [](long long x) { return (x + 31) & ~31LL; };
    const long long np = sw_np(n);
    return al((long long)n * d) + al(np) + np * np + 2 * np * kSwNb + kSwNb * kSwNb + 32 + kSwNb * kSwNb;
}

struct SsPtrs {
    // acc[0] = log det, acc[1] = failure column (as double), acc[2] the pair kernel's
    // arrival counter, acc[4] = y . alpha (sw_pairs_final), acc[8 ..] diagnostics, acc[16 + i] / acc[18 + i] the look-ahead's
    // log det / failure slots; P, P2: the look-ahead's P^-1 buffers (Pg(k & 1))
    double *xs, *alpha, *A, *C0, *C1, *P, *acc, *P2;
    __device__ double* C(int k) const { return (k & 1) ? C1 : C0; }
    __device__ double* Pg(int i) const { return i ? P2 : P; }
};

// The split sweep's launches take a table of thetas (LmlGroup, by value in the
// kernel arguments): each entry carries its own problem (X, y, n), workspace and
// outputs, so one launch set can evaluate the pending L-BFGS-B rounds of several
// concurrent refits (different training sets and n; the same d).  Every theta's
// arithmetic depends only on its own entry -- its work split follows its own n,
// and launch dimensions sized for the largest n only add workgroups that exit --
// so a theta gives the same bits alone, in a batch or grouped with other problems.
constexpr int kMaxGroup = 40;
struct LmlTheta {
    const double* X;          // [n][d]
    const double* y;          // [n]
    const double* theta;      // [d+2] device copy (written by the build from theta_src when set)
    const double* theta_src;  // [d+2] pinned host (device view) or nullptr
    double* lml;              // [1]
    double* grad;             // [d+2]
    int32_t* info;            // [1]
    double* ws;               // ss_ws_doubles(n, d)
    double* partials;         // [kPairGroups][DP + 2]
    int n;
    int pad_;
};
struct LmlGroup {
    int d, count, stop, pad_;
    LmlTheta th[kMaxGroup];
};
// passed by value: the whole table must fit the 4 KiB kernel-argument segment (with the
// launches' other arguments); raising kMaxGroup or growing LmlTheta must keep this
static_assert(sizeof(LmlGroup) + 64 <= 4096, "LmlGroup exceeds the kernel-argument segment");

__device__ __forceinline__ SsPtrs ss_ptrs_t(const LmlTheta& t, int d) {
    auto al = [](long long x) { return (x + 31) & ~31LL; };
    const long long np = sw_np(t.n);
    SsPtrs p;
    p.xs = t.ws;
    p.alpha = p.xs + al((long long)t.n * d);
    p.A = p.alpha + al(np);
    p.C0 = p.A + np * np;
    p.C1 = p.C0 + np * kSwNb;
    p.P = p.C1 + np * kSwNb;
    p.acc = p.P + kSwNb * kSwNb;
    p.P2 = p.acc + 32;
    return p;
}

template <int DP>
__device__ __forceinline__ void ss_theta_p(const double* th, int d, double& amp, double& noise, double (&ls)[DP]) {
    amp = exp(th[0]);
    noise = exp(th[d + 1]);
#pragma unroll
    for (int c = 0; c < DP; ++c) ls[c] = c < d ? exp(th[1 + c]) : 1.0;
}

template <int DP>
__device__ __forceinline__ void ss_theta_t(const LmlTheta& t, int d, double& amp, double& noise, double (&ls)[DP],
                                           bool src) {
    const double* th = src && t.theta_src ? t.theta_src : t.theta;
    amp = exp(th[0]);
    noise = exp(th[d + 1]);
#pragma unroll
    for (int c = 0; c < DP; ++c) ls[c] = c < d ? exp(th[1 + c]) : 1.0;
}

// grid (1, B): xs = X / ls, the log det / failure accumulators
template <int DP>
__global__ __launch_bounds__(256) void sw_xs_kernel(LmlGroup grp) {
    const int b = blockIdx.y;
    const LmlTheta& T = grp.th[b];
    const SsPtrs p = ss_ptrs_t(T, grp.d);
    double amp, noise, ls[DP];
    ss_theta_t<DP>(T, grp.d, amp, noise, ls, false);
    for (int e = threadIdx.x; e < T.n * grp.d; e += blockDim.x) {
        const int c = e % grp.d;
        double lc = 1.0;
#pragma unroll
        for (int q = 0; q < DP; ++q)
            if (q == c) lc = ls[q];
        p.xs[e] = T.X[e] / lc;
    }
    if (threadIdx.x == 0) { p.acc[0] = 0.0; p.acc[1] = 0.0; }
}

// grid (np/16, B): K rows [16 bx, 16 bx + 16) -- the lower triangle and the full
// diagonal 16x16 tiles, identity on the padding
template <int DP>
__global__ __launch_bounds__(256) void sw_build_kernel(LmlGroup grp) {
    const int b = blockIdx.y;
    const LmlTheta& T = grp.th[b];
    const int n = T.n, d = grp.d, np = (int)sw_np(n);
    if ((int)blockIdx.x >= np / 16) return;   // a larger problem of the group sized the grid
    const SsPtrs p = ss_ptrs_t(T, grp.d);
    double amp, noise, ls[DP];
    ss_theta_t<DP>(T, grp.d, amp, noise, ls, false);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int i = 16 * blockIdx.x + wave; i < 16 * blockIdx.x + 16; i += 4) {
        double xi[DP];
#pragma unroll
        for (int c = 0; c < DP; ++c) xi[c] = (c < d && i < n) ? p.xs[i * d + c] : 0.0;
        const int jend = (i | 15) + 1;
        for (int j = lane; j < jend && j < np; j += 64) {
            double v;
            if (i >= n || j >= n) {
                v = i == j ? 1.0 : 0.0;
            } else if (i == j) {
                v = amp * 1.0 + noise + kFitJitter;
            } else {
                double r2 = 0.0;
#pragma unroll
                for (int c = 0; c < DP; ++c)
                    if (c < d) {
                        const double t = xi[c] - p.xs[j * d + c];
                        r2 += t * t;
                    }
                const double k = sqrt(r2) * kSqrt5;
                v = amp * ((1.0 + k + k * k / 3.0) * exp(-k));
            }
            p.A[(long long)i * np + j] = v;
            // C_0 (block column 0 before sweep 0, row-major [np][32]) from the lower
            // entries, as the pivot kernel once copied it out of A
            if (j < kSwNb && j <= i) {
                p.C0[(long long)i * kSwNb + j] = v;
                if (i < kSwNb) p.C0[(long long)j * kSwNb + i] = v;
            }
        }
    }
}

// grid (np/16, B), 1024 threads, dynamic LDS (16 bx + 16) x DP doubles: sw_xs_kernel
// and sw_build_kernel in one launch.  The workgroup divides the X rows its K rows
// need into the LDS (the same X / ls division as sw_xs_kernel), writes its own 16
// rows of xs for the pair kernel, and builds K rows [16 bx, 16 bx + 16) one row per
// wave with sw_build_kernel's arithmetic (the same bits).  Workgroup 0 resets the
// log det / failure accumulators and the pair kernel's arrival counter.
template <int DP>
__global__ __launch_bounds__(1024) void sw_xs_build_kernel(LmlGroup grp) {
    extern __shared__ __attribute__((aligned(16))) double xsl[];   // [rows][DP]
    const int b = blockIdx.y;
    const LmlTheta& T = grp.th[b];
    const int n = T.n, d = grp.d, np = (int)sw_np(n);
    if ((int)blockIdx.x >= np / 16) return;   // a larger problem of the group sized the grid
    const SsPtrs p = ss_ptrs_t(T, grp.d);
    // host-staged call: theta straight from pinned memory, read once per workgroup (one
    // PCIe read per value, not one per wave) and shared through the LDS; workgroup 0
    // writes the device copy the later kernels read
    // The X rows are loaded first, so that their latency overlaps the theta read (the
    // fused build runs only while rows * d <= np * DP <= 8192: at most 8 per thread).
    __shared__ double thl[34];
    const int rows = min(n, 16 * (int)blockIdx.x + 16);
    constexpr int kXPer = 8;
    double xv[kXPer];
#pragma unroll
    for (int u = 0; u < kXPer; ++u) {
        const int e = threadIdx.x + u * 1024;
        xv[u] = e < rows * d ? T.X[e] : 0.0;
    }
    if (threadIdx.x < d + 2) {
        const double v = T.theta_src ? T.theta_src[threadIdx.x] : T.theta[threadIdx.x];
        thl[threadIdx.x] = v;
        if (T.theta_src && blockIdx.x == 0) const_cast<double*>(T.theta)[threadIdx.x] = v;
    }
    __syncthreads();
    double amp, noise, ls[DP];
    ss_theta_p<DP>(thl, grp.d, amp, noise, ls);
#pragma unroll
    for (int u = 0; u < kXPer; ++u) {
        const int e = threadIdx.x + u * 1024;
        if (e >= rows * d) break;
        const int i = e / d, c = e % d;
        double lc = 1.0;
#pragma unroll
        for (int q = 0; q < DP; ++q)
            if (q == c) lc = ls[q];
        const double v = xv[u] / lc;
        xsl[i * DP + c] = v;
        if (i >= 16 * (int)blockIdx.x) p.xs[e] = v;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        p.acc[0] = 0.0;
        p.acc[1] = 0.0;
        *reinterpret_cast<unsigned*>(p.acc + 2) = 0u;
        if (grp.stop == 24) {   // diagnostics only: sw_step_kernel's timestamps (step_stamps)
            unsigned long long* st = reinterpret_cast<unsigned long long*>(p.acc + 8);
            st[0] = ~0ULL; st[1] = 0; st[2] = ~0ULL; st[3] = 0; st[6] = 0;
        }
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int i = 16 * blockIdx.x + wave;
    double xi[DP];
#pragma unroll
    for (int c = 0; c < DP; ++c) xi[c] = (c < d && i < n) ? xsl[i * DP + c] : 0.0;
    const int jend = (i | 15) + 1;
    for (int j = lane; j < jend && j < np; j += 64) {
        double v;
        if (i >= n || j >= n) {
            v = i == j ? 1.0 : 0.0;
        } else if (i == j) {
            v = amp * 1.0 + noise + kFitJitter;
        } else {
            double r2 = 0.0;
#pragma unroll
            for (int c = 0; c < DP; ++c)
                if (c < d) {
                    const double t = xi[c] - xsl[j * DP + c];
                    r2 += t * t;
                }
            const double k = sqrt(r2) * kSqrt5;
            v = amp * ((1.0 + k + k * k / 3.0) * exp(-k));
        }
        p.A[(long long)i * np + j] = v;
        if (j < kSwNb && j <= i) {
            p.C0[(long long)i * kSwNb + j] = v;
            if (i < kSwNb) p.C0[(long long)j * kSwNb + i] = v;
        }
    }
}

// grid (ntile (ntile + 1) / 2, B), 256 threads (r06): sw_xs_build_kernel's work as one
// lower 16x16 tile (I, J) of K per workgroup -- every workgroup divides only its 32 X
// rows by the length scales, and the row-tiled form's last workgroup no longer
// evaluates a whole 16-row band on one CU.  Each element is formed by the same
// expression from the same xs values (the same bits); the diagonal tiles write the xs
// rows for the later kernels, tile (0, 0) the accumulators and the theta device copy.
template <int DP>
__global__ __launch_bounds__(256) void sw_xs_build_tile_kernel(LmlGroup grp) {
    const int b = blockIdx.y;
    const LmlTheta& T = grp.th[b];
    const int n = T.n, d = grp.d, np = (int)sw_np(n), ntile = np / 16;
    const int t = blockIdx.x;
    if (t >= ntile * (ntile + 1) / 2) return;   // a larger problem of the group sized the grid
    int I = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
    while (I * (I + 1) / 2 > t) --I;
    while ((I + 1) * (I + 2) / 2 <= t) ++I;
    const int J = t - I * (I + 1) / 2;
    const SsPtrs p = ss_ptrs_t(T, grp.d);
    __shared__ double thl[34];
    __shared__ double xsl[2][16][DP];   // xs rows 16 I .., 16 J ..
    // the two row blocks' X first (their latency overlaps the theta read)
    const int e0 = threadIdx.x, half = 16 * DP;   // 256 threads cover 2 x 16 x DP <= 1024 elements in 4 passes
    double xv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int e = e0 + 256 * u, w = e / half, r = (e % half) / DP, c = e % DP;
        const int row = 16 * (w ? J : I) + r;
        xv[u] = (e < 2 * half && c < d && row < n) ? T.X[(long long)row * d + c] : 0.0;
    }
    if (threadIdx.x < d + 2) {
        const double v = T.theta_src ? T.theta_src[threadIdx.x] : T.theta[threadIdx.x];
        thl[threadIdx.x] = v;
        if (T.theta_src && t == 0) const_cast<double*>(T.theta)[threadIdx.x] = v;
    }
    if (t == 0 && threadIdx.x == 0) {
        p.acc[0] = 0.0;
        p.acc[1] = 0.0;
        *reinterpret_cast<unsigned*>(p.acc + 2) = 0u;
        if (grp.stop == 24) {   // diagnostics only: sw_step_kernel's timestamps (step_stamps)
            unsigned long long* st = reinterpret_cast<unsigned long long*>(p.acc + 8);
            st[0] = ~0ULL; st[1] = 0; st[2] = ~0ULL; st[3] = 0; st[6] = 0;
        }
        if (grp.stop == 25) {   // diagnostics only: sw_pairs_final_kernel's timestamps
            unsigned long long* st = reinterpret_cast<unsigned long long*>(p.acc + 20);
            st[0] = ~0ULL; st[1] = 0; st[2] = 0; st[3] = 0; st[4] = 0;
        }
    }
    __syncthreads();
    double amp, noise, ls[DP];
    ss_theta_p<DP>(thl, grp.d, amp, noise, ls);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int e = e0 + 256 * u, w = e / half, r = (e % half) / DP, c = e % DP;
        if (e >= 2 * half) break;
        double lc = 1.0;
#pragma unroll
        for (int q = 0; q < DP; ++q)
            if (q == c) lc = ls[q];
        const int row = 16 * (w ? J : I) + r;
        const double v = (c < d && row < n) ? xv[u] / lc : 0.0;
        xsl[w][r][c] = v;
        if (w == 0 && I == J && c < d && row < n) p.xs[(long long)row * d + c] = v;
    }
    __syncthreads();
    const int r = threadIdx.x >> 4, cc = threadIdx.x & 15;
    const int i = 16 * I + r, j = 16 * J + cc;
    double v;
    if (i >= n || j >= n) {
        v = i == j ? 1.0 : 0.0;
    } else if (i == j) {
        v = amp * 1.0 + noise + kFitJitter;
    } else {
        double r2 = 0.0;
#pragma unroll
        for (int c = 0; c < DP; ++c)
            if (c < d) {
                const double tt = xsl[0][r][c] - xsl[1][cc][c];
                r2 += tt * tt;
            }
        const double k = sqrt(r2) * kSqrt5;
        v = amp * ((1.0 + k + k * k / 3.0) * exp(-k));
    }
    p.A[(long long)i * np + j] = v;
    if (j < kSwNb && j <= i) {
        p.C0[(long long)i * kSwNb + j] = v;
        if (i < kSwNb) p.C0[(long long)j * kSwNb + i] = v;
    }
}

// 1 / x for the pivot sweep's serial chain: v_rcp_f64 and two Newton steps (a few
// fp64 FMAs instead of the IEEE division's scale / fixup sequence; within an ulp).
// LML launch 3-4% shorter at n = 128-512 (profiles/r05/fit_pivot_rcp_ab_ag.log)
__device__ __forceinline__ double pivot_rcp(double x) {
    double r = __builtin_amdgcn_rcp(x);
    double e = fma(-x, r, 1.0);
    r = fma(r, e, r);
    e = fma(-x, r, 1.0);
    return fma(r, e, r);
}

// Gauss-Jordan sweep of the 32x32 pivot block rows k0 .. k0+31 of C (row-major
// [np][32]), eliminating with the pivot row (not the symmetric column: that measured
// 10-100x less accurate at cond(K) ~ 1e5).  Two steps per LDS round: the pivot rows c
// and c + 1 are broadcast together, and every lane forms row c + 1 after step c itself
// (row2' = fma(-t21, row1, row2), its column c = t21, pv2 = row2'[c + 1]) and the
// column-(c+1) entry of its own row after step c (colv2' = fma(f1, row1[c+1], colv2),
// 0 for the zeroed pivot row) with exactly the operations the owning lanes perform in
// a one-step sweep (r03: the same bits, tested against it before that form was
// removed) -- half the LDS round trips and serial latency chains, 16 more FMAs per two
// steps.  On return r holds -P^-1 (the lane's columns of its row), prod the product of
// the pivots, bad the first non-positive pivot (1-based) or 0.  A zeroed pivot row is
// written as exec-masked v_mov_b64 (a branch): as plain stores the compiler
// if-converts the branch into two v_cndmask_b32 per double.
//
// The sweep on NW waves (2, 4 or 8): wave w's lane l + 32 h holds the CW =
// 16 / NW columns [16 h + CW w, 16 h + CW w + CW) of row l, so each lane issues 1 / NW
// of the FMAs.  Every element sees exactly the operations of the one-wave form (the
// pivot rows and the pivot columns' entries go through the LDS instead of a cross-lane
// shuffle), so the bits are the same.  One barrier per two sweep steps (the LDS rounds
// alternate between two buffers).  rowb: [2][64] doubles, colb: [2][64].
template <int CW>
__device__ __forceinline__ void zero_cols(double (&r)[CW]) {
#pragma unroll
    for (int jj = 0; jj < CW; ++jj) asm volatile("v_mov_b64 %0, 0" : "=v"(r[jj]));
}

template <int NW>
__device__ __forceinline__ void pivot_block_sweep_nw(const double* __restrict__ C, int k0, double* rowb, double* colb,
                                                     int w, double (&r)[16 / NW], double& prod, int& bad) {
    constexpr int CW = 16 / NW;
    const int lane = threadIdx.x & 63;
    const int l = lane & 31, h = lane >> 5;
    const int col0 = 16 * h + CW * w;   // this lane's first column
#pragma unroll
    for (int jj = 0; jj < CW; ++jj) r[jj] = C[(long long)(k0 + l) * kSwNb + col0 + jj];
    prod = 1.0;
    bad = 0;
#pragma unroll
    for (int c = 0; c < kSwNb; c += 2) {
        double* rb = rowb + ((c >> 1) & 1) * 64;
        double* cl = colb + ((c >> 1) & 1) * 64;
        const int hc = c >> 4, wc = (c & 15) / CW, jc = c % CW;   // columns c, c + 1: one lane's, jc even
        if (h == hc && w == wc) {
            cl[2 * l] = r[jc];           // A[l][c]
            cl[2 * l + 1] = r[jc + 1];   // A[l][c+1], before step c
        }
        const bool piv1 = l == c, piv2 = l == c + 1;
        if (piv1 || piv2) {
#pragma unroll
            for (int jj = 0; jj < CW; ++jj) rb[32 * (l - c) + col0 + jj] = r[jj];
        }
        if (piv1) zero_cols<CW>(r);
        __syncthreads();
        const double colv1 = cl[2 * l], colv2 = cl[2 * l + 1];
        // ---- step c
        const double pv1 = rb[c];
        if (!(pv1 > 0.0) || !isfinite(pv1)) bad = bad ? bad : c + 1;
        prod *= pv1;
        const double ip1 = pivot_rcp(pv1);
        const double t1 = colv1 * ip1;
        const double f1 = piv1 ? ip1 : -t1;
        const double p1c1 = rb[c + 1], p2c = rb[32 + c], p2c1 = rb[32 + c + 1];
        double q1[CW], q2[CW];
#pragma unroll
        for (int jj = 0; jj < CW; ++jj) {
            q1[jj] = rb[col0 + jj];
            q2[jj] = rb[32 + col0 + jj];
        }
        const double t21 = p2c * ip1;
#pragma unroll
        for (int jj = 0; jj < CW; ++jj) {
            const double u = fma(-t21, q1[jj], q2[jj]);
            q2[jj] = col0 + jj == c ? t21 : u;
        }
        const double pv2 = fma(-t21, p1c1, p2c1);
        const double colv2p = fma(f1, p1c1, piv1 ? 0.0 : colv2);
#pragma unroll
        for (int jj = 0; jj < CW; ++jj) {
            const double upd = fma(f1, q1[jj], r[jj]);
            r[jj] = col0 + jj == c ? (piv1 ? -ip1 : t1) : upd;
        }
        // ---- step c + 1 (pivot row = q2)
        if (!(pv2 > 0.0) || !isfinite(pv2)) bad = bad ? bad : c + 2;
        prod *= pv2;
        const double ip2 = pivot_rcp(pv2);
        const double t2 = colv2p * ip2;
        const double f2 = piv2 ? ip2 : -t2;
        if (piv2) zero_cols<CW>(r);
#pragma unroll
        for (int jj = 0; jj < CW; ++jj) {
            const double upd = fma(f2, q2[jj], r[jj]);
            r[jj] = col0 + jj == c + 1 ? (piv2 ? -ip2 : t2) : upd;
        }
        asm volatile("" ::: "memory");
    }
}

// grid (nwg, B), 64 NW threads, nwg * NW * tpw >= the lower tile count: the whole sweep
// step k in one launch.  Every workgroup sweeps the 32x32 pivot block of C_k itself
// (pivot_block_sweep_nw on its NW waves: the same instructions on the same data, so
// the same P^-1 bits in every workgroup) into its LDS while its waves' first tile
// operands land; then each wave forms G_I = C_I P^-1 (16 MFMAs, turned into the
// A-operand layout through its LDS slice) and updates its tile -- tpw tiles per wave,
// tiles t, t + NW nwg, ...; the diagonal tile (I, I) also writes G_I into block column
// k of A (and row I's entries of C_{k+1}), tile (I, I) of block k writes -P^-1 there.
// Workgroup 0 keeps the log det and the failure column.  A tile's arithmetic does not
// depend on which wave computes it, so tpw changes no bits: it trades latency (one
// tile per wave: the step is the sweep plus one update) for fewer redundant sweeps
// when a grouped launch carries many thetas (launch_split_group).
// r05: the sweep on 4 waves instead of 1 (bit-identical): an LML round of 3 thetas
// 166 -> 153 us at n = 256, 316 -> 288 us at n = 448; 2 waves measured the same as 4
// (profiles/r05/lml_sweep2w_ab_a.log, lml_sweep4w_ab_a.log)
__device__ __forceinline__ void step_tile_of(int t, int nt_low, int k, int& I, int& J, int& kind) {
    I = J = kind = 0;   // kind 0: nothing, 1: rows of block k <- -P^-1, 2: update tile (I, J)
    if (t < nt_low) {
        I = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
        while (I * (I + 1) / 2 > t) --I;
        while ((I + 1) * (I + 2) / 2 <= t) ++I;
        J = t - I * (I + 1) / 2;
        kind = (I >> 1) == k ? (I == J ? 1 : 0) : ((J >> 1) == k ? 0 : 2);
    }
    I = __builtin_amdgcn_readfirstlane(I);
    J = __builtin_amdgcn_readfirstlane(J);
    kind = __builtin_amdgcn_readfirstlane(kind);
}

// MPO_FIT_DEBUG=24 (diagnostics only): step 2 of theta 0 records, in its acc[8 ..]
// words, the first / last workgroup entry and exit (wall clock, 100 MHz), workgroup
// 0's shader cycles to the end of the sweep and from there to its exit, and step 1's
// last exit -- the launch gap, the dispatch spread and the sweep's share of a step
__device__ __forceinline__ void step_stamp(const LmlGroup& grp, const SsPtrs& p, int k, int at) {
    if (grp.stop != 24 || blockIdx.y != 0 || (threadIdx.x & 255) != 0) return;
    unsigned long long* st = reinterpret_cast<unsigned long long*>(p.acc + 8);
    const unsigned long long t = wall_clock64();
    if (k == 1 && at == 2) atomicMax(st + 6, t);
    if (k != 2) return;
    if (at == 0) { atomicMin(st + 0, t); atomicMax(st + 1, t); }
    if (at == 2) { atomicMin(st + 2, t); atomicMax(st + 3, t); }
}

// One lower 16x16 tile's update A_IJ -= G_I C_J^T with G_I = C_I P^-1 (16 MFMAs,
// turned into the A-operand layout through the wave's LDS slice g, which keeps G_I
// for the caller); av / cb: rows 16 I / 16 J of C_k in MFMA operand order.
__device__ __forceinline__ void tile_update(const double (&av)[8], const double (&cb)[8], f64x4& acc,
                                            const double* Pl, double* g, int lane) {
    {
        double b0[8], b1[8];
        const double* br = Pl + (lane >> 4) * kSwNb + (lane & 15);
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) {
            b0[ks] = br[4 * ks * kSwNb];
            b1[ks] = br[4 * ks * kSwNb + 16];
        }
        f64x4 acc0 = {0.0, 0.0, 0.0, 0.0}, acc1 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) {
            acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(av[ks], b0[ks], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(av[ks], b1[ks], acc1, 0, 0, 0);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int rr = (lane >> 4) + 4 * q, c0 = lane & 15, c1 = 16 + c0;
            g[(c0 >> 2) * 64 + rr + 16 * (c0 & 3)] = acc0[q];
            g[(c1 >> 2) * 64 + rr + 16 * (c1 & 3)] = acc1[q];
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the wave's G_I stores (LDS ops of one wave complete in order)
    double ga[8];
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) ga[ks] = g[ks * 64 + lane];
#pragma unroll
    for (int ks = 0; ks < 8; ++ks)
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(-ga[ks], cb[ks], acc, 0, 0, 0);
}

// The pivot sweep of rows row0 .. row0 + 31 of src (row-major [.][32]: C_k in global
// memory, or the look-ahead's LDS copy of a diagonal block) on all NW waves of the
// workgroup; -P^-1 lands in dst[32][32] (LDS or global), thread 0 returns the product
// of the pivots and the first bad one.
template <int NW>
__device__ __forceinline__ void sweep_block(const LmlGroup& grp, const double* src, int row0, double* rowb,
                                            double* colb, double* dst, double& prod, int& bad) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    constexpr int CW = 16 / NW;
    const int l = lane & 31, h = lane >> 5, col0 = 16 * h + CW * wv;
    double r[CW];
    if (grp.stop == 23) {   // diagnostics only (MPO_FIT_DEBUG=23): the sweep skipped, timing of the rest
        prod = 1.0;
        bad = 0;
#pragma unroll
        for (int jj = 0; jj < CW; ++jj) r[jj] = src[(long long)(row0 + l) * kSwNb + col0 + jj];
    } else {
        pivot_block_sweep_nw<NW>(src, row0, rowb, colb, wv, r, prod, bad);
    }
#pragma unroll
    for (int jj = 0; jj < CW; ++jj) dst[l * kSwNb + col0 + jj] = -r[jj];
}

// grid (nwg [+ 1], B), 64 NW threads: sweep step k.  LA (look-ahead, r06): the extra first
// workgroup computes the three lower tiles of block k + 1's diagonal block with this
// step's update (tile_update: the same instructions as the workgroups that write them,
// so the same bits), sweeps that block from LDS and writes P_{k+1}^-1 (ws Pg[(k+1)&1])
// and its log det / failure slot; the other workgroups of step k > 0 then load P_k^-1
// instead of sweeping it.  The serial sweep leaves every other workgroup's path, and a
// step ends with the look-ahead's sweep instead of (sweep + update + the slowest
// workgroup's tail).  The first tile workgroup adds the slots to the log det in step
// order (the same sum as before).  Step 0 still sweeps P_0 in every workgroup.
template <bool LA, int NW>
__global__ __launch_bounds__(64 * NW) void sw_step_kernel(LmlGroup grp, int k) {
    const int b = blockIdx.y;
    const LmlTheta& T = grp.th[b];
    const int np = (int)sw_np(T.n), ntile = np / 16, k0 = k * kSwNb;
    if (k0 >= np) return;                     // this problem has fewer pivot blocks
    const SsPtrs p = ss_ptrs_t(T, grp.d);
    step_stamp(grp, p, k, 0);
    const long long c_enter = grp.stop == 24 ? clock64() : 0;
    const double* Cc = p.C(k);
    __shared__ double gl[NW][16 * kSwNb];                 // per wave: G_I, A-operand order
    __shared__ double Pl[kSwNb * kSwNb];                  // P^-1 of this step
    __shared__ double rowb[2 * 2 * kSwNb];
    __shared__ double colb[2 * 2 * kSwNb];
    const int k1 = k0 + kSwNb;
    double* Cn = k1 < np ? p.C(k + 1) : nullptr;
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    double* g = gl[wv];
    if (LA && blockIdx.x == 0) {
        // ---- the look-ahead workgroup (dispatched first): P_{k+1}^-1
        __shared__ double Dl[LA ? kSwNb * kSwNb : 1];     // C_{k+1}'s diagonal block
        if (k1 >= np) return;
        double prod;
        int bad;
        const int I = 2 * k + 2 + (wv > 0), J = 2 * k + 2 + (wv == 2);
        double av[8], cb[8];
        f64x4 acc = {0.0, 0.0, 0.0, 0.0};
        if (wv < 3) {
            const double* ar = Cc + (long long)(16 * I + (lane & 15)) * kSwNb + (lane >> 4);
            const double* cr = Cc + (long long)(16 * J + (lane & 15)) * kSwNb + (lane >> 4);
#pragma unroll
            for (int ks = 0; ks < 8; ++ks) {
                av[ks] = ar[4 * ks];
                cb[ks] = cr[4 * ks];
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[q] = p.A[(long long)(16 * I + (lane >> 4) + 4 * q) * np + 16 * J + (lane & 15)];
        }
        if (k == 0) {
            sweep_block<NW>(grp, Cc, k0, rowb, colb, Pl, prod, bad);
        } else {
            const double* pg = p.Pg((k) & 1);
            for (int e = threadIdx.x; e < kSwNb * kSwNb; e += 64 * NW) Pl[e] = pg[e];
        }
        __syncthreads();
        if (wv < 3) {
            tile_update(av, cb, acc, Pl, g, lane);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int i = 16 * I + (lane >> 4) + 4 * q - k1, j = 16 * J + (lane & 15) - k1;
                if (i < j) continue;                                    // upper half of a diagonal tile
                Dl[i * kSwNb + j] = acc[q];
                Dl[j * kSwNb + i] = acc[q];
            }
        }
        __syncthreads();
        sweep_block<NW>(grp, Dl, 0, rowb, colb, p.Pg((k + 1) & 1), prod, bad);
        if (threadIdx.x == 0) {
            p.acc[16 + ((k + 1) & 1)] = log(prod);
            p.acc[18 + ((k + 1) & 1)] = (double)bad;
        }
        return;
    }
    const int nt_low = ntile * (ntile + 1) / 2;
    const int wg = (int)blockIdx.x - (LA ? 1 : 0);       // this workgroup among the tile workgroups
    const int stride = ((int)gridDim.x - (LA ? 1 : 0)) * NW;
    int t = __builtin_amdgcn_readfirstlane(wg * NW + wv);
    int I, J, kind;
    step_tile_of(t, nt_low, k, I, J, kind);
    // the tile's operands that do not depend on P^-1, loaded while the sweep runs
    // (or P^-1 arrives)
    double av[8], cb[8];
    f64x4 acc = {0.0, 0.0, 0.0, 0.0};
    auto load_tile = [&]() {
        if (kind != 2) return;
        const double* ar = Cc + (long long)(16 * I + (lane & 15)) * kSwNb + (lane >> 4);
        const double* cr = Cc + (long long)(16 * J + (lane & 15)) * kSwNb + (lane >> 4);
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) {
            av[ks] = ar[4 * ks];
            cb[ks] = cr[4 * ks];
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[q] = p.A[(long long)(16 * I + (lane >> 4) + 4 * q) * np + 16 * J + (lane & 15)];
    };
    load_tile();
    if (!LA || k == 0) {
        double prod;
        int bad;
        sweep_block<NW>(grp, Cc, k0, rowb, colb, Pl, prod, bad);
        if (wg == 0 && threadIdx.x == 0) {
            p.acc[0] += log(prod);
            if (bad && p.acc[1] == 0.0) p.acc[1] = (double)(k0 + bad);
        }
    } else {
        const double* pg = p.Pg(k & 1);
        for (int e = threadIdx.x; e < kSwNb * kSwNb; e += 64 * NW) Pl[e] = pg[e];
        if (wg == 0 && threadIdx.x == 0) {
            p.acc[0] += p.acc[16 + (k & 1)];
            const int bad = (int)p.acc[18 + (k & 1)];
            if (bad && p.acc[1] == 0.0) p.acc[1] = (double)(k0 + bad);
        }
    }
    __syncthreads();
    const long long c_swept = grp.stop == 24 ? clock64() : 0;
    for (;;) {
        if (kind == 1) {
#pragma unroll
            for (int e = lane; e < 16 * kSwNb; e += 64) {
                const int i = 16 * I + (e >> 5), c = e & 31;
                p.A[(long long)i * np + k0 + c] = -Pl[(i - k0) * kSwNb + c];
            }
        } else if (kind == 2) {
            tile_update(av, cb, acc, Pl, g, lane);
            // with the look-ahead, block k + 1's diagonal tiles are not stored to A: those
            // stores are dead (step k + 1 overwrites the block with -P^-1) and the
            // look-ahead workgroup of this step reads the block's step-k input there
            if (!LA || (I >> 1) != k + 1 || (J >> 1) != k + 1) {
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    p.A[(long long)(16 * I + (lane >> 4) + 4 * q) * np + 16 * J + (lane & 15)] = acc[q];
            }
            if (Cn && ((J >> 1) == k + 1 || (I >> 1) == k + 1)) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int i = 16 * I + (lane >> 4) + 4 * q, j = 16 * J + (lane & 15);
                    if (i < j) continue;                                    // upper half of a diagonal tile
                    if ((j >> 5) == k + 1) Cn[(long long)i * kSwNb + (j - k1)] = acc[q];
                    if ((i >> 5) == k + 1) Cn[(long long)j * kSwNb + (i - k1)] = acc[q];
                }
            }
            if (I == J) {
                // block column k, rows 16 I .. 16 I + 15, <- G_I (lower storage: below
                // block k at A[i][j], above it transposed at A[j][i]); a row of block k+1
                // also gives row j of C_{k+1}
#pragma unroll
                for (int e = lane; e < 16 * kSwNb; e += 64) {
                    const int ri = e >> 5, c = e & 31, i = 16 * I + ri, j = k0 + c;
                    const double gv = g[(c >> 2) * 64 + ri + 16 * (c & 3)];
                    if (i > j) p.A[(long long)i * np + j] = gv;
                    else p.A[(long long)j * np + i] = gv;
                    if (Cn && (i >> 5) == k + 1) Cn[(long long)j * kSwNb + (i - k1)] = gv;
                }
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // g's reads before the next tile's stores
        }
        t += stride;
        if (t >= nt_low) break;
        step_tile_of(t, nt_low, k, I, J, kind);
        acc = f64x4{0.0, 0.0, 0.0, 0.0};
        load_tile();
    }
    if (grp.stop == 24) {
        step_stamp(grp, p, k, 2);
        if (k == 2 && wg == 0 && blockIdx.y == 0 && threadIdx.x == 0) {
            unsigned long long* st = reinterpret_cast<unsigned long long*>(p.acc + 8);
            st[4] = (unsigned long long)(c_swept - c_enter);
            st[5] = (unsigned long long)(clock64() - c_swept);
        }
    }
}

// grid (np/16, B), 256 threads: alpha = K^-1 y for the 16 rows of row tile I;
// wave w sums the column tiles J = w (mod 4), each tile read from the lower
// storage (transposed above the diagonal); fixed-order reductions.  The J loop
// unrolled by 4 lets the loads run ahead of the fma chain (same order; 7.95 -> 6.89 us
// at n = 448, profiles/r05/lml_alpha_unroll_a.log)
__global__ __launch_bounds__(256) void sw_alpha_kernel(LmlGroup grp) {
    __shared__ double part[4][16];
    const int b = blockIdx.y;
    const LmlTheta& T = grp.th[b];
    const int n = T.n, np = (int)sw_np(n), ntile = np / 16, I = blockIdx.x;
    if (I >= ntile) return;
    const SsPtrs p = ss_ptrs_t(T, grp.d);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = lane & 15, cq = lane >> 4;
    const int i = 16 * I + r;
    double sacc = 0.0;
#pragma unroll 4
    for (int J = wave; J < ntile; J += 4) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int j = 16 * J + cq + 4 * u;
            const double kij = j <= i ? -p.A[(long long)i * np + j] : -p.A[(long long)j * np + i];
            sacc = fma(kij, j < n ? T.y[j] : 0.0, sacc);
        }
    }
    sacc += __shfl_xor(sacc, 16);
    sacc += __shfl_xor(sacc, 32);
    if (cq == 0) part[wave][r] = sacc;
    __syncthreads();
    if (threadIdx.x < 16) {
        const int ii = 16 * I + threadIdx.x;
        const double v = (part[0][threadIdx.x] + part[1][threadIdx.x]) + (part[2][threadIdx.x] + part[3][threadIdx.x]);
        p.alpha[ii] = ii < n ? v : 0.0;
    }
}

// per-theta partial gradients of the pair kernel: [kPairGroups][DP + 2] after the
// workspace's own end (mpo_gp_lml_ws_bytes adds them)
constexpr int kPairGroups = 64;

// The pairs i >= j of rows i = gw, gw + nw, ... (one wave per row): W_ij dK_ij/dtheta
// (sklearn kernels.py:1747-1767) into g, each lane taking j = lane, lane + 64, ...
// Two pairs' operands (alpha_j, A_ij, xs_j) are loaded before either is evaluated, so
// one load latency covers two pairs; the lane still adds its pairs in j order
// (bit-identical; sw_pairs_final 22.4 -> 19.2 us at n = 448, profiles/r05/lml_pair_prefetch_a.log).
template <int DP>
__device__ __forceinline__ void pair_rows(const SsPtrs& p, int n, int d, int np, double amp, double noise, int gw,
                                          int nw, int lane, double (&g)[DP + 2]) {
    for (int i = gw; i < n; i += nw) {
        const double ai = p.alpha[i];
        double xi[DP];
#pragma unroll
        for (int c = 0; c < DP; ++c) xi[c] = c < d ? p.xs[i * d + c] : 0.0;
        for (int j0 = lane; j0 <= i; j0 += 128) {
            double aj[2], aij[2], xj[2][DP];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int j = j0 + 64 * u <= i ? j0 + 64 * u : j0;
                aj[u] = p.alpha[j];
                aij[u] = p.A[(long long)i * np + j];
#pragma unroll
                for (int c = 0; c < DP; ++c) xj[u][c] = c < d ? p.xs[j * d + c] : 0.0;
            }
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int j = j0 + 64 * u;
                if (j > i) break;
                const double W = (ai * aj[u] + aij[u]) * (i == j ? 1.0 : 2.0);
                double r2 = 0.0;
#pragma unroll
                for (int c = 0; c < DP; ++c)
                    if (c < d) {
                        const double t = xi[c] - xj[u][c];
                        r2 += t * t;
                    }
                const double sq = sqrt(5.0 * r2);
                const double e = exp(-sq);
                const double Mij = i == j ? 1.0 : (1.0 + sq + sq * sq / 3.0) * e;
                g[0] += W * (amp * Mij);
                const double f = W * amp * (5.0 / 3.0) * (sq + 1.0) * e;
#pragma unroll
                for (int c = 0; c < DP; ++c)
                    if (c < d) {
                        const double t = xi[c] - xj[u][c];
                        g[1 + c] += f * (t * t);
                    }
                if (i == j) g[DP + 1] += W * noise;
            }
        }
    }
}

// grid (kPairGroups, B), 256 threads: pairs i >= j of rows i = gw (mod waves),
// W_ij dK_ij/dtheta; one partial per workgroup
template <int DP>
__global__ __launch_bounds__(256) void sw_pairs_kernel(LmlGroup grp) {
    __shared__ double red[4][DP + 2];
    const int b = blockIdx.y;
    const LmlTheta& T = grp.th[b];
    const int n = T.n, d = grp.d, np = (int)sw_np(n);
    const SsPtrs p = ss_ptrs_t(T, grp.d);
    double amp, noise, ls[DP];
    ss_theta_t<DP>(T, grp.d, amp, noise, ls, false);
    (void)ls;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int gw = blockIdx.x * 4 + wave, nw = gridDim.x * 4;
    double g[DP + 2];
#pragma unroll
    for (int c = 0; c < DP + 2; ++c) g[c] = 0.0;
    if (p.acc[1] == 0.0) pair_rows<DP>(p, n, d, np, amp, noise, gw, nw, lane, g);
#pragma unroll
    for (int c = 0; c < DP + 2; ++c) {
        const double v = wave_sum_bcast(g[c]);
        if (lane == 0) red[wave][c] = v;
    }
    __syncthreads();
    if (threadIdx.x < DP + 2) {
        const int c = threadIdx.x;
        T.partials[(long long)blockIdx.x * (DP + 2) + c] = (red[0][c] + red[1][c]) + (red[2][c] + red[3][c]);
    }
}

// grid (1, B), 64 threads: y.alpha, the LML, the gradient from the pair partials
// (fixed order), or sklearn's LinAlgError branch (-inf, zeros)
template <int DP>
__global__ __launch_bounds__(64) void sw_final_kernel(LmlGroup grp, int groups) {
    const int b = blockIdx.y;
    const LmlTheta& T = grp.th[b];
    const int n = T.n, d = grp.d, lane = threadIdx.x;
    const SsPtrs p = ss_ptrs_t(T, grp.d);
    double* out = T.grad;
    if (p.acc[1] != 0.0) {
        if (lane == 0) { T.lml[0] = -INFINITY; T.info[0] = (int)p.acc[1]; }
        for (int c = lane; c < d + 2; c += 64) out[c] = 0.0;
        return;
    }
    double ya = 0.0;
    for (int i = lane; i < n; i += 64) ya = fma(T.y[i], p.alpha[i], ya);
    ya = wave_sum_bcast(ya);
    if (lane == 0) {
        T.lml[0] = -0.5 * ya - 0.5 * p.acc[0] - 0.5 * n * kLog2Pi;
        T.info[0] = 0;
    }
    if (lane < d + 2) {
        const int src = lane == 0 ? 0 : (lane == d + 1 ? DP + 1 : lane);
        double sum = 0.0;
        for (int w = 0; w < groups; ++w) sum += T.partials[(long long)w * (DP + 2) + src];
        out[lane] = 0.5 * sum;
    }
}

// sw_pairs_kernel + sw_final_kernel in one launch: every workgroup stores its
// partial, then the last one to arrive (a device-scope counter per theta, reset by
// sw_xs_build_kernel) sums the partials -- loaded in parallel into the LDS, then
// added in sw_final_kernel's fixed order -- and writes y.alpha, the LML and the
// gradient (the same bits as the two-launch form).
template <int DP>
__global__ __launch_bounds__(256) void sw_pairs_final_kernel(LmlGroup grp) {
    __shared__ double red[4][DP + 2];
    __shared__ double pl[kPairGroups * (DP + 2)];
    __shared__ int last;
    const int b = blockIdx.y;
    const LmlTheta& T = grp.th[b];
    const int n = T.n, d = grp.d, np = (int)sw_np(n);
    const SsPtrs p = ss_ptrs_t(T, grp.d);
    double amp, noise, ls[DP];
    ss_theta_t<DP>(T, grp.d, amp, noise, ls, false);
    (void)ls;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int gw = blockIdx.x * 4 + wave, nw = gridDim.x * 4;
    // MPO_FIT_DEBUG=25 (diagnostics only): theta 0's entry spread, pairs done, tail start / end
    unsigned long long* pst = reinterpret_cast<unsigned long long*>(p.acc + 20);
    const bool stamp = grp.stop == 25 && blockIdx.y == 0 && threadIdx.x == 0;
    if (stamp) { const unsigned long long t = wall_clock64(); atomicMin(pst + 0, t); atomicMax(pst + 1, t); }
    const bool failed = p.acc[1] != 0.0;
    double g[DP + 2];
#pragma unroll
    for (int c = 0; c < DP + 2; ++c) g[c] = 0.0;
    // y . alpha off the tail: workgroup 0's wave 0 forms it first (the same per-lane fma
    // order and butterfly as the last workgroup once did) and leaves it in acc[4]
    if (blockIdx.x == 0 && wave == 0 && !failed) {
        double ya = 0.0;
        for (int i = lane; i < n; i += 64) ya = fma(T.y[i], p.alpha[i], ya);
        ya = wave_sum_bcast(ya);
        if (lane == 0) p.acc[4] = ya;
    }
    if (!failed) pair_rows<DP>(p, n, d, np, amp, noise, gw, nw, lane, g);
#pragma unroll
    for (int c = 0; c < DP + 2; ++c) {
        const double v = wave_sum_bcast(g[c]);
        if (lane == 0) red[wave][c] = v;
    }
    __syncthreads();
    if (threadIdx.x < DP + 2) {
        const int c = threadIdx.x;
        T.partials[(long long)blockIdx.x * (DP + 2) + c] = (red[0][c] + red[1][c]) + (red[2][c] + red[3][c]);
    }
    __syncthreads();
    if (stamp) atomicMax(pst + 2, wall_clock64());
    if (threadIdx.x == 0) {
        // one device-scope release per workgroup (after the barrier it covers the
        // partial rows written by threads 0 .. DP+1): each fence writes back this
        // XCD's L2, and one per writing thread cost ~4 us per launch
        __threadfence();
        last = atomicAdd(reinterpret_cast<unsigned*>(p.acc + 2), 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (!last) return;
    __threadfence();
    if (stamp) pst[3] = wall_clock64();
    const int groups = gridDim.x;
    double* out = T.grad;
    if (failed) {
        if (threadIdx.x == 0) { T.lml[0] = -INFINITY; T.info[0] = (int)p.acc[1]; }
        for (int c = threadIdx.x; c < d + 2; c += 256) out[c] = 0.0;
        return;
    }
    for (int e = threadIdx.x; e < groups * (DP + 2); e += 256)
        pl[e] = T.partials[e];
    __syncthreads();
    if (wave != 0) return;
    if (lane == 0) {
        const double ya = p.acc[4];
        T.lml[0] = -0.5 * ya - 0.5 * p.acc[0] - 0.5 * n * kLog2Pi;
        T.info[0] = 0;
    }
    if (lane < d + 2) {
        const int src = lane == 0 ? 0 : (lane == d + 1 ? DP + 1 : lane);
        double sum = 0.0;
        for (int w = 0; w < groups; ++w) sum += pl[w * (DP + 2) + src];
        out[lane] = 0.5 * sum;
    }
    if (stamp) pst[4] = wall_clock64();
}

// One evaluation of the thetas th[0 .. count) (any problems of dimension d, DP =
// fit_dp(d)): the split sweep's launches, in chunks of kMaxGroup thetas, the grids
// sized for the chunk's largest n (the smaller problems' extra workgroups exit).
// The fused build / finish while the largest problem's xs rows fit 64 KiB of LDS;
// past it separate xs / build / pairs / final launches (the same arithmetic; those
// read theta from the device copy, so a group there carries no theta_src).
inline int fit_dp(int d);

template <int DP>
int launch_split_group(const LmlTheta* th, int count, int d, int stop, hipStream_t s) {
    for (int c0 = 0; c0 < count; c0 += kMaxGroup) {
        LmlGroup g{};
        g.d = d;
        g.stop = stop;
        g.count = std::min(kMaxGroup, count - c0);
        int nmax = 0;
        for (int i = 0; i < g.count; ++i) {
            g.th[i] = th[c0 + i];
            nmax = std::max(nmax, g.th[i].n);
        }
        const int np = (int)sw_np(nmax), nbk = np / kSwNb, ntile = np / 16, B = g.count;
        const int nt_low = ntile * (ntile + 1) / 2;
        // tiles per wave: one while the launch's workgroups fit ~4 per CU (latency: a step
        // is one sweep plus one tile update); more when a grouped launch carries many
        // thetas, so fewer workgroups repeat the pivot sweep
        static const long long wg_target = [] {   // MPO_FIT_STEP_WG: tuning sweeps only
            const char* e = getenv("MPO_FIT_STEP_WG");
            return e && *e ? std::max(1LL, atoll(e)) : kStepWgTarget;
        }();
        // MPO_FIT_LOOKAHEAD (0 | 1): P_{k+1}^-1 swept by one extra workgroup of step k;
        // MPO_FIT_STEP_WAVES (2 | 4 | 8): waves per step workgroup, all of which share the
        // pivot sweep (the same bits either way)
        static const int lookahead = [] {
            const char* e = getenv("MPO_FIT_LOOKAHEAD");
            return e && *e ? atoi(e) : 1;
        }();
        static const int nw = [] {
            const char* e = getenv("MPO_FIT_STEP_WAVES");
            const int v = e && *e ? atoi(e) : kStepWaves;
            return v == 2 || v == 8 ? v : 4;
        }();
        int tpw = kUpdTilesPerWave;
        while (tpw < 16 && (long long)B * nt_low / ((long long)nw * tpw) > wg_target) tpw *= 2;
        const int nwg = std::max(1, (nt_low + nw * tpw - 1) / (nw * tpw));
        const size_t xs_lds = (size_t)np * DP * sizeof(double);
        const bool fuse_build = xs_lds <= 64 * 1024;   // np * DP <= 8192: sw_xs_build_kernel's 8 X values per thread
        // MPO_FIT_BUILD=rows: the row-band build (one 16-row band per workgroup), for A/B
        static const bool tile_build = [] {
            const char* e = getenv("MPO_FIT_BUILD");
            return !(e && std::string(e) == "rows");
        }();
        if (fuse_build && tile_build) {
            hipLaunchKernelGGL(sw_xs_build_tile_kernel<DP>, dim3(nt_low, B), dim3(256), 0, s, g);
            MPO_LAUNCH_CHECK();
        } else if (fuse_build) {
            auto kb = sw_xs_build_kernel<DP>;
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kb), hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)xs_lds);
            hipLaunchKernelGGL(kb, dim3(ntile, B), dim3(1024), xs_lds, s, g);
            MPO_LAUNCH_CHECK();
        } else {
            for (int i = 0; i < B; ++i)
                if (g.th[i].theta_src) {
                    mpo::set_error("mpo_gp_lml_grad: a host theta source needs the fused split sweep");
                    return MPO_EINVAL;
                }
            hipLaunchKernelGGL(sw_xs_kernel<DP>, dim3(1, B), dim3(256), 0, s, g);
            MPO_LAUNCH_CHECK();
            hipLaunchKernelGGL(sw_build_kernel<DP>, dim3(ntile, B), dim3(256), 0, s, g);
            MPO_LAUNCH_CHECK();
        }
        for (int k = 0; k < nbk; ++k) {
            const dim3 grid(nwg + (lookahead ? 1 : 0), B), block(64 * nw);
            if (lookahead) {
                if (nw == 8) hipLaunchKernelGGL((sw_step_kernel<true, 8>), grid, block, 0, s, g, k);
                else if (nw == 2) hipLaunchKernelGGL((sw_step_kernel<true, 2>), grid, block, 0, s, g, k);
                else hipLaunchKernelGGL((sw_step_kernel<true, 4>), grid, block, 0, s, g, k);
            } else {
                if (nw == 8) hipLaunchKernelGGL((sw_step_kernel<false, 8>), grid, block, 0, s, g, k);
                else if (nw == 2) hipLaunchKernelGGL((sw_step_kernel<false, 2>), grid, block, 0, s, g, k);
                else hipLaunchKernelGGL((sw_step_kernel<false, 4>), grid, block, 0, s, g, k);
            }
            MPO_LAUNCH_CHECK();
        }
        hipLaunchKernelGGL(sw_alpha_kernel, dim3(ntile, B), dim3(256), 0, s, g);
        MPO_LAUNCH_CHECK();
        if (fuse_build) {   // the arrival counter is reset by sw_xs_build_kernel
            hipLaunchKernelGGL(sw_pairs_final_kernel<DP>, dim3(kPairGroups, B), dim3(256), 0, s, g);
            MPO_LAUNCH_CHECK();
        } else {
            hipLaunchKernelGGL(sw_pairs_kernel<DP>, dim3(kPairGroups, B), dim3(256), 0, s, g);
            MPO_LAUNCH_CHECK();
            hipLaunchKernelGGL(sw_final_kernel<DP>, dim3(1, B), dim3(64), 0, s, g, kPairGroups);
            MPO_LAUNCH_CHECK();
        }
    }
    return MPO_OK;
}

// the thetas of one problem (X, y, n): theta / lml / grad / info as mpo_gp_lml_grad
// lays them out, workspace per theta then the pair partials per theta
inline void problem_thetas(std::vector<LmlTheta>& out, const double* X, const double* y, int n, int d, int dp,
                           const double* theta, const double* theta_src, int batch, double* lml, double* grad,
                           int32_t* info, double* ws) {
    const long long stride = ss_ws_doubles(n, d);
    double* partials = ws + (long long)batch * stride;
    for (int b = 0; b < batch; ++b) {
        LmlTheta t{};
        t.X = X;
        t.y = y;
        t.theta = theta + (long long)b * (d + 2);
        t.theta_src = theta_src ? theta_src + (long long)b * (d + 2) : nullptr;
        t.lml = lml + b;
        t.grad = grad + (long long)b * (d + 2);
        t.info = info + b;
        t.ws = ws + (long long)b * stride;
        t.partials = partials + (long long)b * kPairGroups * (dp + 2);
        t.n = n;
        out.push_back(t);
    }
}

int launch_split_any(const std::vector<LmlTheta>& th, int d, int stop, hipStream_t s) {
    switch (fit_dp(d)) {
        case 4: return launch_split_group<4>(th.data(), (int)th.size(), d, stop, s);
        case 8: return launch_split_group<8>(th.data(), (int)th.size(), d, stop, s);
        case 12: return launch_split_group<12>(th.data(), (int)th.size(), d, stop, s);
        case 16: return launch_split_group<16>(th.data(), (int)th.size(), d, stop, s);
        default: return launch_split_group<32>(th.data(), (int)th.size(), d, stop, s);
    }
}

inline int fit_dp(int d) {
    if (d <= 4) return 4;
    if (d <= 8) return 8;
    if (d <= 12) return 12;
    if (d <= 16) return 16;
    if (d <= 32) return 32;
    return -1;
}

// which LML kernel: the LDS-packed Cholesky kernel for n <= kSplitMinN (small,
// latency-bound factors), the split block sweep past it (0.09 vs 0.20 ms at n = 64,
// 0.30 ms at n = 200 against 0.68 for the Cholesky kernel: scripts/fit_probe.py).
// MPO_FIT_KERNEL = panel / split forces one (tests: each kernel outside its range).
// the split sweep: n > kSplitMinN (MPO_FIT_KERNEL=split forces it for n > 16)
inline bool use_split(int n) {
    const char* e = getenv("MPO_FIT_KERNEL");
    if (e && std::string(e) == "split") return n > 16 && n <= kFitMaxN;
    if (e && std::string(e) == "panel" && n <= kFitLdsMaxN) return false;
    return n > kSplitMinN;
}

// the fused split sweep (launch_split's fuse_build): the host-staged call may hand it theta
// and the outputs in pinned host memory
inline bool fit_fused_split(int n, int dp) {
    return use_split(n) && (size_t)sw_np(n) * dp * sizeof(double) <= 64 * 1024;
}

template <bool kLds, int DP>
int launch_lml(const LmlArgs& a, int B, hipStream_t s) {
    auto kern = lml_grad_kernel<kLds, DP>;
    const size_t lds = kLds ? (size_t)fit_tri(a.n) * sizeof(double) : (size_t)kFitWaves * (DP + 2) * sizeof(double);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(kern, dim3(B), dim3(kFitThreads), lds, s, a);
    MPO_LAUNCH_CHECK();
    return MPO_OK;
}

}  // namespace

namespace mpo {

bool lml_groupable(int n, int d) {
    const int dp = fit_dp(d);
    return dp > 0 && n > 0 && n <= kFitMaxN && fit_fused_split(n, dp);
}

int lml_launch_rounds(const LmlRound* r, int count, hipStream_t s) {
    if (count <= 0) return MPO_OK;
    const int d = r[0].d, dp = fit_dp(d), k = d + 2;
    std::vector<LmlTheta> th;
    for (int i = 0; i < count; ++i) {
        MPO_CHECK_ARG(r[i].d == d && lml_groupable(r[i].n, d), "lml_launch_rounds: round %d not groupable", i);
        double* od = r[i].out;
        const int B = r[i].batch;
        problem_thetas(th, r[i].X, r[i].y, r[i].n, d, dp, r[i].theta_dev, r[i].theta_src, B, od, od + B,
                       reinterpret_cast<int32_t*>(od + B + (long long)B * k), r[i].ws);
    }
    return launch_split_any(th, d, 0, s);
}

}  // namespace mpo

extern "C" {

size_t mpo_gp_lml_ws_bytes(int n, int d, int batch) {
    if (n <= 0 || n > kFitMaxN || fit_dp(d) < 0 || batch <= 0) return 0;
    const long long per = std::max(fit_ws_doubles(n, d, n <= kFitLdsMaxN), ss_ws_doubles(n, d));
    return ((size_t)per * batch + (size_t)batch * kPairGroups * 34) * sizeof(double) + 256;   // + pair partials
}

static int lml_grad_impl(const double* X, const double* y_norm, int n, int d, const double* theta,
                         const double* theta_src, int batch, double* lml, double* grad, int32_t* info, void* ws,
                         size_t ws_bytes, void* stream);

int mpo_gp_lml_grad(const double* X, const double* y_norm, int n, int d, const double* theta, int batch,
                    double* lml, double* grad, int32_t* info, void* ws, size_t ws_bytes, void* stream) {
    return lml_grad_impl(X, y_norm, n, d, theta, nullptr, batch, lml, grad, info, ws, ws_bytes, stream);
}

static int lml_grad_impl(const double* X, const double* y_norm, int n, int d, const double* theta,
                         const double* theta_src, int batch, double* lml, double* grad, int32_t* info, void* ws,
                         size_t ws_bytes, void* stream) {
    MPO_GUARD_BEGIN
    MPO_CHECK_ARG(X && y_norm && theta && lml && grad && info && ws, "mpo_gp_lml_grad: null pointer");
    MPO_CHECK_ARG(n > 0 && d > 0 && batch > 0, "mpo_gp_lml_grad: bad shape n=%d d=%d batch=%d", n, d, batch);
    const int dp = fit_dp(d);
    if (dp < 0 || n > kFitMaxN) {
        mpo::set_error("mpo_gp_lml_grad: n=%d d=%d outside n<=%d, d<=32", n, d, kFitMaxN);
        return MPO_ENOTSUP;
    }
    MPO_CHECK_ARG(ws_bytes >= mpo_gp_lml_ws_bytes(n, d, batch), "mpo_gp_lml_grad: workspace too small (%zu < %zu)",
                  ws_bytes, mpo_gp_lml_ws_bytes(n, d, batch));
    const bool use_lds = n <= kFitLdsMaxN;
    const bool split = use_split(n);
    double* wsa = reinterpret_cast<double*>(mpo::align_up(reinterpret_cast<uintptr_t>(ws), 256));
    LmlArgs a{X, y_norm, n, d, theta, lml, grad, info, wsa, fit_ws_doubles(n, d, use_lds), 0};
    int stop = 0;
    if (const char* e = getenv("MPO_FIT_DEBUG")) stop = a.stop = atoi(e);
    a.theta_src = split && fit_fused_split(n, dp) ? theta_src : nullptr;
    MPO_CHECK_ARG(!theta_src || a.theta_src, "mpo_gp_lml_grad: a host theta source needs the fused split sweep");
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (split) {
        std::vector<LmlTheta> th;
        th.reserve(batch);
        problem_thetas(th, X, y_norm, n, d, dp, theta, a.theta_src, batch, lml, grad, info, wsa);
        return launch_split_any(th, d, stop, s);
    }
    if (use_lds) {
        switch (dp) {
            case 4: return launch_lml<true, 4>(a, batch, s);
            case 8: return launch_lml<true, 8>(a, batch, s);
            case 12: return launch_lml<true, 12>(a, batch, s);
            case 16: return launch_lml<true, 16>(a, batch, s);
            default: return launch_lml<true, 32>(a, batch, s);
        }
    }
    switch (dp) {
        case 4: return launch_lml<false, 4>(a, batch, s);
        case 8: return launch_lml<false, 8>(a, batch, s);
        case 12: return launch_lml<false, 12>(a, batch, s);
        case 16: return launch_lml<false, 16>(a, batch, s);
        default: return launch_lml<false, 32>(a, batch, s);
    }
    MPO_GUARD_END
}

size_t mpo_gp_lml_io_bytes(int d, int batch) {
    if (d <= 0 || batch <= 0) return 0;
    const size_t k = (size_t)d + 2;
    return ((size_t)batch * k + (size_t)batch + (size_t)batch * k + ((size_t)batch + 1) / 2) * sizeof(double);
}

int mpo_gp_lml_grad_host(const double* X, const double* y_norm, int n, int d, const double* theta_host, int batch,
                         double* out_host, void* dev_io, size_t io_bytes, void* ws, size_t ws_bytes, void* stream) {
    MPO_GUARD_BEGIN
    MPO_CHECK_ARG(theta_host && out_host && dev_io, "mpo_gp_lml_grad_host: null pointer");
    mpo::StreamDeviceScope on_device(static_cast<hipStream_t>(stream));
    MPO_CHECK_ARG(d > 0 && batch > 0, "mpo_gp_lml_grad_host: bad shape d=%d batch=%d", d, batch);
    MPO_CHECK_ARG(io_bytes >= mpo_gp_lml_io_bytes(d, batch), "mpo_gp_lml_grad_host: io buffer too small (%zu < %zu)",
                  io_bytes, mpo_gp_lml_io_bytes(d, batch));
    const size_t k = (size_t)d + 2;
    double* th = static_cast<double*>(dev_io);
    double* out = th + (size_t)batch * k;                  // lml | grad | info, as out_host
    double* lml = out;
    double* grad = out + batch;
    int32_t* info = reinterpret_cast<int32_t*>(grad + (size_t)batch * k);
    hipStream_t s = static_cast<hipStream_t>(stream);
    // Pinned host buffers on the fused split sweep: the first kernel reads theta from
    // the host copy and the last writes lml | grad | info straight into out_host --
    // no copy launches around the round (two of ~20 launches, ~7 us at n = 256).
    const int dp = fit_dp(d);
    if (dp > 0 && fit_fused_split(n, dp)) {
        hipPointerAttribute_t ta{}, oa{};
        if (hipPointerGetAttributes(&ta, theta_host) == hipSuccess && ta.type == hipMemoryTypeHost && ta.devicePointer &&
            hipPointerGetAttributes(&oa, out_host) == hipSuccess && oa.type == hipMemoryTypeHost && oa.devicePointer) {
            double* od = static_cast<double*>(oa.devicePointer);
            const int rc = lml_grad_impl(X, y_norm, n, d, th, static_cast<const double*>(ta.devicePointer), batch, od,
                                         od + batch, reinterpret_cast<int32_t*>(od + batch + (size_t)batch * k), ws,
                                         ws_bytes, stream);
            if (rc != MPO_OK) return rc;
            MPO_HIP(hipStreamSynchronize(s));
            return MPO_OK;
        }
        (void)hipGetLastError();   // an unregistered pointer: the copies below
    }
    MPO_HIP(hipMemcpyAsync(th, theta_host, (size_t)batch * k * sizeof(double), hipMemcpyHostToDevice, s));
    const int rc = mpo_gp_lml_grad(X, y_norm, n, d, th, batch, lml, grad, info, ws, ws_bytes, stream);
    if (rc != MPO_OK) return rc;
    const size_t out_bytes = ((size_t)batch + (size_t)batch * k + ((size_t)batch + 1) / 2) * sizeof(double);
    MPO_HIP(hipMemcpyAsync(out_host, out, out_bytes, hipMemcpyDeviceToHost, s));
    MPO_HIP(hipStreamSynchronize(s));
    return MPO_OK;
    MPO_GUARD_END
}

}  // extern "C"
