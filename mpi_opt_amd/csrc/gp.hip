// gp.hip -- fp64 GP posterior + acquisition scoring for gfx950 (MI355X).
//
// Hot path G1-G4 of SURVEY §8a: the skopt "ask" step.  The reference reaches it
// through Coordinator.fit/ask (/root/reference/coordinator.py:63-79, 46-50) ->
// skopt.Optimizer -> GaussianProcessRegressor.predict + gaussian_ei/pi/lcb.
//
// Kernels
//   scale_rows_kernel    xs = X / ls (dims zero-padded to DP)
//   kernel_matrix_kernel K  = amp * Matern52(|xs_i - xs_j|) + diag
//   chol_kernel          in-place lower Cholesky (one workgroup)
//   trsm_kernel          L X = B / L^T X = B, one thread per right-hand side
//   pack_wfrag_kernel    L^-1 -> MFMA B-fragment stream (lower triangle only)
//   gp_score_kernel      per 16/32/64-candidate block:
//                          phase 1 (VALU): K*[m][i] = Matern52 into LDS in MFMA
//                                          A-fragment order, mu partials
//                          phase 2 (MFMA): V = K* . L^-T on v_mfma_f64_16x16x4,
//                                          only the lower-triangular k-steps,
//                                          ||V_row||^2 accumulated in registers
//                          phase 3:        sd, mu, -EI/-PI/LCB, block top-k
//   topk_merge_kernel    block top-k partials -> global top-k (lowest index ties)
//
// Why the triangular form: skopt evaluates sd^2 = amp - k^T K_inv k with an
// explicit K_inv (86 kFLOP/candidate at N=200, catastrophic cancellation);
// sd^2 = amp - ||L^-1 k||^2 is the same posterior with half the MFMA work and
// ~1000x less rounding error (DESIGN.md "GP posterior formulation").

#include "mpo_internal.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <string>

namespace {

typedef double f64x4 __attribute__((ext_vector_type(4)));

constexpr double kSqrt5 = 2.236067977499789696409173668731276235;
constexpr double kSqrt1_2 = 0.707106781186547524400844362104849039;
constexpr double kSqrt2Pi = 2.506628274631000502415765284811045253;
constexpr double kJitter = 1e-10;
  // sklearn GPR alpha default (_gpr.py:207)

// sklearn kernels.py:1715-1724 (nu = 2.5) times ConstantKernel.
__device__ __forceinline__ double matern52(double r, double amp) {
    // k^2 / 3 as a multiply by the rounded 1/3: within 1 ulp of sklearn's division,
    // and an fp64 divide costs ~10 VALU ops per candidate-observation pair
    const double k = r * kSqrt5;
    return amp * ((1.0 + k + k * k * (1.0 / 3.0)) * exp(-k));
}

// exp(-k) for k >= 0 without the generic exp's special-case handling (k is a
// scaled distance: never negative, never NaN): Cody-Waite reduction
// k = n ln2 + r, |r| <= ln2/2, degree-13 Taylor polynomial of exp(-r) (truncation
// < 4e-18 relative), 2^-n by ldexp.  k is clamped at 800 (exp(-800) underflows to
// exactly 0, as the padding rows need).  Within 2 ulp of exp(-k).
__device__ __forceinline__ double exp_neg(double k) {
    k = fmin(k, 800.0);
    const double t = rint(k * 1.44269504088896340736);
    const double r = fma(-t, 1.90821492927058770002e-10, fma(-t, 6.93147180369123816490e-01, k));
    const double x = -r;
    double p = 1.0 / 6227020800.0;                  // 1/13!
    p = fma(p, x, 1.0 / 479001600.0);
    p = fma(p, x, 1.0 / 39916800.0);
    p = fma(p, x, 1.0 / 3628800.0);
    p = fma(p, x, 1.0 / 362880.0);
    p = fma(p, x, 1.0 / 40320.0);
    p = fma(p, x, 1.0 / 5040.0);
    p = fma(p, x, 1.0 / 720.0);
    p = fma(p, x, 1.0 / 120.0);
    p = fma(p, x, 1.0 / 24.0);
    p = fma(p, x, 1.0 / 6.0);
    p = fma(p, x, 0.5);
    p = fma(p, x, 1.0);
    p = fma(p, x, 1.0);
    return ldexp(p, -(int)t);
}

// sqrt of a non-negative finite r2 by v_rsq_f64, a Goldschmidt step and one
// Newton correction (ocml's sequence without its denormal scaling and 0/inf
// fix-ups: r2 is clamped below at 1e-300, whose square root 1e-150 gives the same
// Matern value as 0).  Within 2 ulp; an ulp of r moves K* by <= 1e-14 relative.
__device__ __forceinline__ double sqrt_pos(double r2) {
    r2 = fmax(r2, 1e-300);
    const double y = __builtin_amdgcn_rsq(r2);
    double s = r2 * y, h = 0.5 * y;
    const double e0 = fma(-h, s, 0.5);
    s = fma(s, e0, s);
    h = fma(h, e0, h);
    const double e1 = fma(-s, s, r2);
    return fma(e1, h, s);
}

// The scoring kernel's Matern WITHOUT the ConstantKernel amplitude:
// (1 + k + k^2/3) exp(-k), k = sqrt(5 r2), k^2/3 = r2 * 5/3.  The kernel folds amp
// into mu (amp * K'.alpha) and into q (amp^2 ||L^-1 K'||^2): one multiply fewer per
// candidate-observation pair -- fp64 VALU and fp64 MFMA work do not overlap on
// gfx950 (scripts/probes/coexec.hip), so every VALU op per pair is kernel time.
__device__ __forceinline__ double matern52_unit(double r2) {
    const double k = sqrt_pos(r2) * kSqrt5;
    return fma(r2, 5.0 / 3.0, 1.0 + k) * exp_neg(k);
}

// scipy.special.ndtr (cephes ndtr.c), the kernel of scipy.stats.norm.cdf.
__device__ __forceinline__ double ndtr(double a) {
    const double x = a * kSqrt1_2;
    const double z = fabs(x);
    if (z < kSqrt1_2) return 0.5 + 0.5 * erf(x);
    double y = 0.5 * erfc(z);
    return x > 0.0 ? 1.0 - y : y;
}

__device__ __forceinline__ double norm_pdf(double x) { return exp(-x * x / 2.0) / kSqrt2Pi; }

// (value, index) lexicographic order: smaller value first, lower index on ties.
__device__ __forceinline__ bool lex_less(double v, long long i, double w, long long j) {
    return v < w || (v == w && i < j);
}

__device__ __forceinline__ void wave_lex_min(double& v, long long& i) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        double w = __shfl_xor(v, off);
        long long j = __shfl_xor(i, off);
        if (lex_less(w, j, v, i)) { v = w; i = j; }
    }
}

// Rows [n, rows) are padding: a point 1e30 away in every real dimension, whose
// Matern value underflows to exactly 0 (and alpha is 0 there): a scoring loop may
// run over whole 32-observation groups without bounds checks.
constexpr double kFarAway = 1e30;

__global__ void scale_rows_kernel(const double* __restrict__ X, int n, int rows, int d, int dp,
                                  const double* __restrict__ ls, double* __restrict__ xs,
                                  double* __restrict__ ls_pad) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < rows * dp) {
        const int i = t / dp, c = t % dp;
        xs[t] = c < d ? (i < n ? X[(size_t)i * d + c] / ls[c] : kFarAway) : 0.0;
    }
    if (ls_pad && t < dp) ls_pad[t] = t < d ? ls[t] : 1.0;
}

__global__ void zero_kernel(double* __restrict__ p, int n) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n) p[t] = 0.0;
}

__global__ void kernel_matrix_kernel(const double* __restrict__ xs, int n, int dp, double amp,
                                     double diag_add, double* __restrict__ K, int ldk) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    const int i = blockIdx.y;
    if (j >= n) return;
    double r2 = 0.0;
    for (int c = 0; c < dp; ++c) {
        const double t = xs[(size_t)i * dp + c] - xs[(size_t)j * dp + c];
        r2 += t * t;
    }
    double v = matern52(sqrt(r2), amp);
    if (i == j) v += diag_add;
    K[(size_t)i * ldk + j] = v;
}

// K from unscaled X (mpo_gp_kernel_matrix has no workspace for xs): divides
// by ls inline, like sklearn's pdist(X / length_scale).
__global__ void kernel_matrix_unscaled_kernel(const double* __restrict__ X, int n, int d,
                                              const double* __restrict__ ls, double amp,
                                              double diag_add, double* __restrict__ K, int ldk) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    const int i = blockIdx.y;
    if (j >= n) return;
    double r2 = 0.0;
    for (int c = 0; c < d; ++c) {
        const double t = X[(size_t)i * d + c] / ls[c] - X[(size_t)j * d + c] / ls[c];
        r2 += t * t;
    }
    double v = matern52(sqrt(r2), amp);
    if (i == j) v += diag_add;
    K[(size_t)i * ldk + j] = v;
}

// Right-looking unblocked Cholesky in one workgroup; A stays in global memory
// (L2-resident at the sizes skopt reaches).  Off the per-candidate hot path:
// run once per GP refit.
__global__ __launch_bounds__(1024) void chol_kernel(double* __restrict__ A, int n, int lda,
                                                    int32_t* __restrict__ info) {
    __shared__ int fail;
    const int tid = threadIdx.x, nt = blockDim.x;
    const int lane = tid & 63, wave = tid >> 6, nwave = nt >> 6;
    if (tid == 0) fail = 0;
    __syncthreads();
    for (int j = 0; j < n; ++j) {
        if (tid == 0) {
            const double djj = A[(size_t)j * lda + j];
            if (!(djj > 0.0) || !isfinite(djj)) fail = j + 1;
            else A[(size_t)j * lda + j] = sqrt(djj);
        }
        __syncthreads();
        if (fail) break;
        const double ljj = A[(size_t)j * lda + j];
        for (int i = j + 1 + tid; i < n; i += nt) A[(size_t)i * lda + j] /= ljj;
        __syncthreads();
        for (int i = j + 1 + wave; i < n; i += nwave) {
            const double lij = A[(size_t)i * lda + j];
            for (int k = j + 1 + lane; k <= i; k += 64)
                A[(size_t)i * lda + k] -= lij * A[(size_t)k * lda + j];
        }
        __syncthreads();
    }
    if (tid == 0) *info = fail;
}

// One thread per right-hand-side column; the solution vector lives in LDS
// ([n][cb], conflict-free across the cb columns of a block).
__global__ __launch_bounds__(64) void trsm_kernel(const double* __restrict__ L, int n, int lda,
                                                  double* __restrict__ B, int nrhs, int ldb,
                                                  int trans, int cb) {
    extern __shared__ __attribute__((aligned(16))) double xsol[];
    const int lc = threadIdx.x;
    const int col = blockIdx.x * cb + lc;
    const bool active = lc < cb && col < nrhs;
    if (!active) return;
    if (!trans) {
        for (int i = 0; i < n; ++i) {
            double s = B[(size_t)i * ldb + col];
            const double* Li = L + (size_t)i * lda;
            for (int k = 0; k < i; ++k) s -= Li[k] * xsol[k * cb + lc];
            const double x = s / Li[i];
            xsol[i * cb + lc] = x;
            B[(size_t)i * ldb + col] = x;
        }
    } else {
        for (int i = n - 1; i >= 0; --i) {
            double s = B[(size_t)i * ldb + col];
            for (int k = i + 1; k < n; ++k) s -= L[(size_t)k * lda + i] * xsol[k * cb + lc];
            const double x = s / L[(size_t)i * lda + i];
            xsol[i * cb + lc] = x;
            B[(size_t)i * ldb + col] = x;
        }
    }
}

__global__ void fill_identity_kernel(double* __restrict__ W, int n, int ldw) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    const int i = blockIdx.y;
    if (j < n) W[(size_t)i * ldw + j] = (i == j) ? 1.0 : 0.0;
}

__global__ void copy_kernel(const double* __restrict__ src, double* __restrict__ dst, int n) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n) dst[t] = src[t];
}

// B-fragment stream of W^T (W = L^-1 lower): column tile jt of 16 columns needs
// the k-steps ks < 4(jt+1) (rows i <= 16 jt + 15); lane l of k-step ks holds
// W^T[4 ks + (l>>4)][16 jt + (l&15)] = W[16 jt + (l&15)][4 ks + (l>>4)].
__host__ __device__ constexpr size_t wfrag_tile_base(int jt) { return (size_t)128 * jt * (jt + 1); }
inline size_t wfrag_elems(int np16) { return wfrag_tile_base(np16 / 16) + 16 * 64; }  // + prefetch slack

__global__ void pack_wfrag_kernel(const double* __restrict__ W, int n, int ldw, int T,
                                  double* __restrict__ wfrag) {
    const int jt = blockIdx.y;
    if (jt >= T) return;
    const int nks = 4 * (jt + 1);
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= nks * 64) return;
    const int ks = e >> 6, l = e & 63;
    const int i = 4 * ks + (l >> 4), j = 16 * jt + (l & 15);
    const double v = (i < n && j < n && i <= j) ? W[(size_t)j * ldw + i] : 0.0;
    wfrag[wfrag_tile_base(jt) + e] = v;
}

// ---------------------------------------------------------------------------
struct ScoreArgs {
    int n, np16, T, d;
    double amp, y_mean, y_std;
    const double* xs;
    const double* ls;
    const double* alpha;
    const double* wfrag;
    const double* cand;
    long long m;
    double y_opt, xi, kappa;
    unsigned flags;
    int ei_positive;  // write +EI (mpo_gp_ei_score) instead of -EI into vals
    double* mu;
    double* sd;
    double* vals;
    int k;
    long long* part_idx;  // [nblocks][3][k]
    double* part_val;
};

// Posterior, acquisitions and the tile's top-k from mu_n = K* alpha and
// q = ||L^-1 k*||^2 of one candidate per lane (``live`` lanes own a row).
__device__ __forceinline__ void score_epilogue(const ScoreArgs& a, bool live, long long gm, double mu_n, double q,
                                               long long part, int lane) {
    const bool valid = live && gm < a.m;
    double mu = 0.0, sd = 0.0, vei = 0.0, vpi = 0.0, vlcb = 0.0;
    if (live) {
        double var = a.amp - q;
        if (var < 0.0) var = 0.0;
        sd = sqrt(var) * a.y_std;
        mu = a.y_std * mu_n + a.y_mean;
        if (sd > 0.0) {
            const double improve = a.y_opt - a.xi - mu;
            const double scaled = improve / sd;
            const double cdf = ndtr(scaled);
            vei = -(improve * cdf + sd * norm_pdf(scaled));
            vpi = -cdf;
        } else {
            vei = -0.0;
            vpi = -0.0;
        }
        vlcb = mu - a.kappa * sd;
    }
    if (valid) {
        if (a.mu) a.mu[gm] = mu;
        if (a.sd) a.sd[gm] = sd;
        if (a.vals) {
            if (a.flags & MPO_ACQ_EI) a.vals[gm] = a.ei_positive ? -vei : vei;
            if (a.flags & MPO_ACQ_PI) a.vals[a.m + gm] = vpi;
            if (a.flags & MPO_ACQ_LCB) a.vals[2 * a.m + gm] = vlcb;
        }
    }
    if (a.k > 0) {
        const double inf = __builtin_huge_val();
#pragma unroll
        for (int acq = 0; acq < 3; ++acq) {
            if (!(a.flags & (1u << acq))) continue;
            double v = valid ? (acq == 0 ? vei : (acq == 1 ? vpi : vlcb)) : inf;
            long long idx = valid ? gm : 0x7fffffffffffffffLL;
            long long* pi = a.part_idx + ((size_t)part * 3 + acq) * a.k;
            double* pv = a.part_val + ((size_t)part * 3 + acq) * a.k;
            for (int r = 0; r < a.k; ++r) {
                double bv = v;
                long long bi = idx;
                wave_lex_min(bv, bi);
                if (lane == 0) { pv[r] = bv; pi[r] = bi; }
                if (idx == bi) { v = inf; idx = 0x7fffffffffffffffLL; }
            }
        }
    }
}

template <int BM, int DP, int D, int OCC>
__global__ __launch_bounds__(256, OCC) void gp_score_kernel(ScoreArgs a) {
    constexpr int MT = BM / 16;      // 16-row m-tiles per block
    constexpr int G = 64 / BM;       // lanes groups per wave in phase 1
    constexpr int S = 4 * G;         // i-slots per block in phase 1
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int np16 = a.np16;
    double* kc = smem;                          // [np16/4][MT][64]
    double* cs = kc + (size_t)np16 * BM;        // [BM][DP]
    double* red = cs + BM * DP;                 // [S][BM] (mu) then [4][BM] (q)

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const long long m0 = (long long)blockIdx.x * BM;

    // ---- phase 0: candidate tile / ls -> LDS
    for (int e = tid; e < BM * DP; e += 256) {
        const int r = e / DP, c = e % DP;
        const long long gm = m0 + r;
        cs[e] = (gm < a.m && c < a.d) ? a.cand[gm * a.d + c] / a.ls[c] : 0.0;
    }
    __syncthreads();

    // ---- phase 1: K*[row][i] (Matern52) in A-fragment order, mu partials
    {
        const int row = lane % BM;
        const int slot = wave * G + lane / BM;
        double c[DP];
#pragma unroll
        for (int q = 0; q < DP; ++q) c[q] = cs[row * DP + q];
        double mu_acc = 0.0;
        const int kc_row = (row >> 4) * 64 + (row & 15);
        for (int i = slot; i < np16; i += S) {
            double kv = 0.0;
            if (i < a.n) {
                const double* xi_ = a.xs + (size_t)i * DP;
                double r2 = 0.0;
#pragma unroll
                for (int q = 0; q < D; ++q) {      // D real dims of the DP-padded rows
                    const double t = c[q] - xi_[q];
                    r2 += t * t;
                }
                kv = matern52_unit(r2);             // amp folded into mu and q below
                mu_acc += kv * a.alpha[i];
            }
            kc[(size_t)((i >> 2) * MT) * 64 + kc_row + (i & 3) * 16] = kv;
        }
        red[slot * BM + row] = mu_acc;
    }
    __syncthreads();
    double mu_n = 0.0;
    if (tid < BM) {
#pragma unroll
        for (int s = 0; s < S; ++s) mu_n += red[s * BM + tid];
        mu_n *= a.amp;
    }
    __syncthreads();  // red is reused for the q partials below

    // ---- phase 2: V = K* L^-T on f64 MFMA, lower-triangular k-steps only
    {
        double sq[MT][4];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int r = 0; r < 4; ++r) sq[mt][r] = 0.0;
        const int T = a.T;
        for (int p = 0; p < T; ++p) {
            const int q8 = p & 7;
            const int owner = q8 < 4 ? q8 : 7 - q8;  // snake over descending tile cost
            if (owner != wave) continue;
            const int jt = T - 1 - p;
            const double* bp = a.wfrag + wfrag_tile_base(jt) + lane;
            const int nks = 4 * (jt + 1);
            // CH independent accumulation chains per m-tile (k-step mod CH) hide
            // the f64 MFMA dependency latency: 4 chains at one m-tile per wave.
            constexpr int CH = 2;   // 4 chains at MT = 1 measured slower (1.94 vs 1.68 ms / 1M)
            f64x4 acc[MT][CH];
#pragma unroll
            for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                for (int c = 0; c < CH; ++c) acc[mt][c] = f64x4{0.0, 0.0, 0.0, 0.0};
            // nks is a multiple of 4.  B fragments stream from L2 two 4-k-step groups
            // ahead (8 MFMAs ~ the L2 latency); slots past the tile read the next
            // tile's fragments (wfrag has 8 k-steps of slack at its end), unused.
            double bq[2][4];
#pragma unroll
            for (int g = 0; g < 2; ++g)
#pragma unroll
                for (int u = 0; u < 4; ++u) bq[g][u] = bp[(4 * g + u) * 64];
            for (int ks = 0; ks < nks; ks += 8) {
#pragma unroll
                for (int g = 0; g < 2; ++g) {
                    if (ks + 4 * g >= nks) break;
                    const double* ap = kc + (size_t)(ks + 4 * g) * MT * 64 + lane;
                    double cur[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        cur[u] = bq[g][u];
                        bq[g][u] = bp[(ks + 8 + 4 * g + u) * 64];
                    }
#pragma unroll
                    for (int u = 0; u < 4; ++u)
#pragma unroll
                        for (int mt = 0; mt < MT; ++mt)
                            acc[mt][u % CH] = __builtin_amdgcn_mfma_f64_16x16x4f64(ap[(u * MT + mt) * 64], cur[u],
                                                                                 acc[mt][u % CH], 0, 0, 0);
                }
            }
#pragma unroll
            for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    double v = acc[mt][0][r];
#pragma unroll
                    for (int c = 1; c < CH; ++c) v += acc[mt][c][r];
                    sq[mt][r] += v * v;
                }
        }
        // f64 C/D map: col = lane & 15, row = (lane >> 4) + 4 r.  Sum the columns.
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                double v = sq[mt][r];
                v += __shfl_xor(v, 1);
                v += __shfl_xor(v, 2);
                v += __shfl_xor(v, 4);
                v += __shfl_xor(v, 8);
                if ((lane & 15) == 0) red[wave * BM + mt * 16 + (lane >> 4) + 4 * r] = v;
            }
    }
    __syncthreads();

    // ---- phase 3: posterior, acquisitions, block top-k (wave 0)
    if (wave != 0) return;
    const int row = lane;
    const double q = row < BM ? (red[0 * BM + row] + red[1 * BM + row] + red[2 * BM + row] + red[3 * BM + row]) *
                                    (a.amp * a.amp) : 0.0;
    score_epilogue(a, row < BM, m0 + row, mu_n, q, blockIdx.x, lane);
}

// Merge per-block top-k lists.  grid = (G, 3): block g of acquisition y merges
// the partial lists [g*chunk, min((g+1)*chunk, nparts)) and writes one list.
// Stage 1 writes the partial layout [(g*3 + acq)*k + r]; the final stage (G = 1)
// writes out[acq*out_stride + r] with index -1 for missing entries.
__global__ __launch_bounds__(256) void topk_merge_kernel(const long long* __restrict__ part_idx,
                                                         const double* __restrict__ part_val,
                                                         int nparts, int chunk, int k, unsigned flags,
                                                         long long* __restrict__ out_idx,
                                                         double* __restrict__ out_val,
                                                         int out_stride, int final_stage) {
    __shared__ double lv[256 * MPO_TOPK_MAX];
    __shared__ long long li[256 * MPO_TOPK_MAX];
    const int acq = blockIdx.y;
    if (!(flags & (1u << acq))) return;
    const int tid = threadIdx.x;
    const double inf = __builtin_huge_val();
    const long long big = 0x7fffffffffffffffLL;
    const int p0 = blockIdx.x * chunk;
    const int p1 = min(nparts, p0 + chunk);
    double bv[MPO_TOPK_MAX];
    long long bi[MPO_TOPK_MAX];
#pragma unroll
    for (int r = 0; r < MPO_TOPK_MAX; ++r) { bv[r] = inf; bi[r] = big; }
    const long long total = (long long)(p1 - p0) * k;
    for (long long e = tid; e < total; e += 256) {
        const long long blk = p0 + e / k, r = e % k;
        const size_t off = ((size_t)blk * 3 + acq) * k + r;
        double v = part_val[off];
        long long i = part_idx[off];
#pragma unroll
        for (int s = 0; s < MPO_TOPK_MAX; ++s) {
            if (s < k && lex_less(v, i, bv[s], bi[s])) {
                const double tv = bv[s];
                const long long ti = bi[s];
                bv[s] = v; bi[s] = i; v = tv; i = ti;
            }
        }
    }
#pragma unroll
    for (int r = 0; r < MPO_TOPK_MAX; ++r) { lv[tid * MPO_TOPK_MAX + r] = bv[r]; li[tid * MPO_TOPK_MAX + r] = bi[r]; }
    __syncthreads();
    if (tid >= 64) return;
    // wave 0: k rounds of a 256-list merge; lane owns lists lane, lane+64, ...
    int ptr[4] = {0, 0, 0, 0};
    for (int r = 0; r < k; ++r) {
        double v = inf;
        long long i = big;
        int src = -1;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int lst = tid + 64 * q;
            if (ptr[q] < k) {
                const double w = lv[lst * MPO_TOPK_MAX + ptr[q]];
                const long long j = li[lst * MPO_TOPK_MAX + ptr[q]];
                if (lex_less(w, j, v, i)) { v = w; i = j; src = q; }
            }
        }
        double gv = v;
        long long gi = i;
        wave_lex_min(gv, gi);
        if (src >= 0 && gi == i && gv == v) {
#pragma unroll
            for (int q = 0; q < 4; ++q) if (q == src) ptr[q]++;
        }
        if (tid == 0) {
            if (final_stage) {
                out_val[acq * out_stride + r] = gv;
                out_idx[acq * out_stride + r] = gi == big ? -1 : gi;
            } else {
                out_val[((size_t)blockIdx.x * 3 + acq) * k + r] = gv;
                out_idx[((size_t)blockIdx.x * 3 + acq) * k + r] = gi;
            }
        }
    }
}

__global__ void argmax_from_topk_kernel(const long long* __restrict__ topk_idx, long long* __restrict__ argmax) {
    *argmax = topk_idx[0];
}

inline int pad_dims(int d) {
    if (d <= 4) return 4;
    if (d <= 8) return 8;
    if (d <= 12) return 12;
    if (d <= 16) return 16;
    if (d <= 32) return 32;
    return -1;
}

constexpr size_t kMaxLds = 160 * 1024;
constexpr int kMergeGroups = 256;  // stage-1 top-k merge groups

size_t score_lds_bytes(int bm, int dp, int np16) {
    const int S = 4 * (64 / bm);
    const int red = std::max(S * bm, 4 * bm);
    return ((size_t)np16 * bm + (size_t)bm * dp + red) * sizeof(double);
}

// Candidates per workgroup.  MPO_GP_BM (16/32/64) overrides the default for
// experiments; the default prefers the variant that fits several workgroups per
// CU (VALU Matern phase of one overlapping the MFMA phase of another).
int choose_bm(int dp, int np16) {
    const char* env = getenv("MPO_GP_BM");
    const int forced = env ? atoi(env) : 0;
    if ((forced == 16 || forced == 32 || forced == 64) && score_lds_bytes(forced, dp, np16) <= kMaxLds) return forced;
    for (int bm : {16, 32, 64})
        if (score_lds_bytes(bm, dp, np16) <= kMaxLds) return bm;
    return -1;
}

template <int BM, int DP, int D, int OCC>
hipError_t launch_score(const ScoreArgs& a, int nblocks, size_t lds, hipStream_t s) {
    auto kern = gp_score_kernel<BM, DP, D, OCC>;
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                        (int)lds);
    hipLaunchKernelGGL(kern, dim3(nblocks), dim3(256), lds, s, a);
    return hipGetLastError();
}

// occupancy hint for the 16-candidate variant (min waves per SIMD -> VGPR cap);
// MPO_GP_OCC overrides for experiments
inline int gp_occ16() {
    const char* e = getenv("MPO_GP_OCC");
    const int v = e ? atoi(e) : 6;
    return (v == 1 || v == 5 || v == 6 || v == 8) ? v : 6;
}

template <int DP, int D>
hipError_t launch_score_bm(int bm, const ScoreArgs& a, int nblocks, size_t lds, hipStream_t s) {
    switch (bm) {
        case 64: return launch_score<64, DP, D, 1>(a, nblocks, lds, s);
        case 32: return launch_score<32, DP, D, 1>(a, nblocks, lds, s);
        case 16:
            switch (gp_occ16()) {
                case 1: return launch_score<16, DP, D, 1>(a, nblocks, lds, s);
                case 5: return launch_score<16, DP, D, 5>(a, nblocks, lds, s);
                case 8: return launch_score<16, DP, D, 8>(a, nblocks, lds, s);
                default: return launch_score<16, DP, D, 6>(a, nblocks, lds, s);
            }
    }
    return hipErrorInvalidValue;
}

// (padded row width DP, distance dims D): d = 5 and d = 10 (the reference's mnist
// space and the BASELINE config) get exact-width distance loops
hipError_t launch_score_dp(int dp, int d, int bm, const ScoreArgs& a, int nblocks, size_t lds, hipStream_t s) {
    switch (dp) {
        case 4: return launch_score_bm<4, 4>(bm, a, nblocks, lds, s);
        case 8: return d == 5 ? launch_score_bm<8, 5>(bm, a, nblocks, lds, s)
                              : launch_score_bm<8, 8>(bm, a, nblocks, lds, s);
        case 12: return d == 10 ? launch_score_bm<12, 10>(bm, a, nblocks, lds, s)
                                : launch_score_bm<12, 12>(bm, a, nblocks, lds, s);
        case 16: return launch_score_bm<16, 16>(bm, a, nblocks, lds, s);
        case 32: return launch_score_bm<32, 32>(bm, a, nblocks, lds, s);
    }
    return hipErrorInvalidValue;
}

constexpr int kWaveTile = 16;   // candidates per partial top-k list (the smallest block)

int trsm_cols_per_block(int n) {
    size_t cb = 64;
    while (cb > 1 && (size_t)n * cb * sizeof(double) > kMaxLds - 1024) cb >>= 1;
    return (int)cb;
}

int trsm_launch(const double* L, int n, int lda, double* B, int nrhs, int ldb, int trans,
                hipStream_t s) {
    const int cb = trsm_cols_per_block(n);
    const size_t lds = (size_t)n * cb * sizeof(double);
    if (lds > kMaxLds) {
        mpo::set_error("mpo_trsm_f64: n=%d too large", n);
        return MPO_ENOTSUP;
    }
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(trsm_kernel),
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(trsm_kernel, dim3((nrhs + cb - 1) / cb), dim3(64), lds, s, L, n, lda, B,
                       nrhs, ldb, trans, cb);
    MPO_LAUNCH_CHECK();
    return MPO_OK;
}

// ---------------------------------------------------------------------------
// Acquisition value + gradient at a few points: the objective of skopt's
// L-BFGS-B polish of the best n_restarts_optimizer candidates per acquisition
// (skopt optimizer.py _tell -> fmin_l_bfgs_b(gaussian_acquisition_1D, ...,
// maxiter=20); gaussian_acquisition_1D / gaussian_ei/pi/lcb(return_grad=True) and
// GaussianProcessRegressor.predict(return_mean_grad, return_std_grad)).  All
// polishes of one ask step run in lockstep, so one launch carries one point per
// live L-BFGS-B run: one workgroup per point, the posterior as in the scoring
// kernel but with the explicit derivative of k* (skopt gpr.py):
//   dk_i/dx_j  = c_i (x_j - X_ij) / ls_j^2,  c_i = -(5/3) amp (1 + t_i) e^-t_i
//   dmu/dx     = y_std dk^T alpha
//   dsd/dx     = -y_std dk^T (W^T W k*) / sd_n,  W = L^-1
// LDS: k*, c (n each), v = W k* (n), four per-wave partials of W^T v (4 n).
constexpr int kGradThreads = 256;

__global__ __launch_bounds__(kGradThreads) void acq_grad_kernel(
        int n, int d, int dp, double amp, double y_mean, double y_std, const double* __restrict__ xs,
        const double* __restrict__ ls, const double* __restrict__ alpha, const double* __restrict__ W,
        const double* __restrict__ x, const int32_t* __restrict__ acq, double y_opt, double xi, double kappa,
        double* __restrict__ f, double* __restrict__ g) {
    extern __shared__ double sm[];
    double* kk = sm;              // [n]
    double* cc = kk + n;          // [n]
    double* vv = cc + n;          // [n]
    double* up = vv + n;          // [4][n]
    __shared__ double xp[32];     // x / ls
    __shared__ double red[kGradThreads];
    __shared__ double ga[8][32], gu[8][32];
    const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid < 32) xp[tid] = tid < d ? x[(size_t)b * d + tid] / ls[tid] : 0.0;
    __syncthreads();

    // k*, c and mu_n partials
    double mu_part = 0.0;
    for (int i = tid; i < n; i += kGradThreads) {
        double r2 = 0.0;
        for (int j = 0; j < d; ++j) {
            const double t = xp[j] - xs[(size_t)i * dp + j];
            r2 = fma(t, t, r2);
        }
        const double t = kSqrt5 * sqrt(r2);
        const double e = exp(-t);
        const double k = amp * ((1.0 + t + t * t * (1.0 / 3.0)) * e);
        kk[i] = k;
        cc[i] = (-5.0 / 3.0) * amp * (1.0 + t) * e;
        mu_part = fma(k, alpha[i], mu_part);
    }
    for (int i = tid; i < 4 * n; i += kGradThreads) up[i] = 0.0;
    __syncthreads();

    // v = W k* (rows per wave, lanes across the row), q = ||v||^2
    double q_part = 0.0;
    for (int r = wave; r < n; r += 4) {
        double s = 0.0;
        for (int c = lane; c <= r; c += 64) s = fma(W[(size_t)r * n + c], kk[c], s);
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off);
        if (lane == 0) vv[r] = s;
        q_part = fma(s, s, q_part);     // identical in every lane: count lane 0 only
    }
    if (lane != 0) q_part = 0.0;
    __syncthreads();

    // u = W^T v: wave w accumulates rows r = w (mod 4) into its own partial
    double* uw = up + (size_t)wave * n;
    for (int r = wave; r < n; r += 4) {
        const double vr = vv[r];
        for (int c = lane; c <= r; c += 64) uw[c] = fma(W[(size_t)r * n + c], vr, uw[c]);
    }
    __syncthreads();
    for (int i = tid; i < n; i += kGradThreads) up[i] = (up[i] + up[n + i]) + (up[2 * n + i] + up[3 * n + i]);

    // block sums of mu_n and q
    red[tid] = mu_part;
    __syncthreads();
    for (int s = kGradThreads / 2; s > 0; s >>= 1) {
        if (tid < s) red[tid] += red[tid + s];
        __syncthreads();
    }
    const double mu_n = red[0];
    __syncthreads();
    red[tid] = q_part;
    __syncthreads();
    for (int s = kGradThreads / 2; s > 0; s >>= 1) {
        if (tid < s) red[tid] += red[tid + s];
        __syncthreads();
    }
    const double q = red[0];

    // dk^T alpha and dk^T u per dimension: thread (grp, j) sums observations grp (mod 8)
    {
        const int j = tid & 31, grp = tid >> 5;
        double sa = 0.0, su = 0.0;
        if (j < d) {
            for (int i = grp; i < n; i += 8) {
                const double t = cc[i] * (xp[j] - xs[(size_t)i * dp + j]);
                sa = fma(t, alpha[i], sa);
                su = fma(t, up[i], su);
            }
        }
        ga[grp][j] = sa;
        gu[grp][j] = su;
    }
    __syncthreads();

    if (tid < d) {
        const int j = tid;
        double sa = 0.0, su = 0.0;
        for (int grp = 0; grp < 8; ++grp) {
            sa += ga[grp][j];
            su += gu[grp][j];
        }
        const double inv_ls = 1.0 / ls[j];
        double var = amp - q;
        if (var < 0.0) var = 0.0;
        const double sd_n = sqrt(var);
        const double mu = y_std * mu_n + y_mean;
        const double sd = sd_n * y_std;
        const double mu_g = y_std * sa * inv_ls;
        const double sd_g = sd_n > 0.0 ? -y_std * su * inv_ls / sd_n : 0.0;
        const int a = acq[b];
        double fv, gv;
        if (a == (int)MPO_ACQ_LCB) {
            fv = mu - kappa * sd;
            gv = mu_g - kappa * sd_g;
        } else if (sd <= 0.0) {
            fv = 0.0;
            gv = 0.0;
        } else {
            const double improve = y_opt - xi - mu;
            const double z = improve / sd;
            const double cdf = ndtr(z), pdf = norm_pdf(z);
            const double improve_g = (-mu_g * sd - sd_g * improve) / (sd * sd);
            if (a == (int)MPO_ACQ_PI) {
                fv = -cdf;
                gv = -(improve_g * pdf);
            } else {
                const double cdf_g = improve_g * pdf;
                const double pdf_g = -improve * cdf_g;
                fv = -(improve * cdf + sd * pdf);
                gv = -((-mu_g * cdf - pdf_g) + (sd_g * pdf + pdf_g));
            }
        }
        g[(size_t)b * d + j] = gv;
        if (j == 0) f[b] = fv;
    }
}

}  // namespace

// ===========================================================================
extern "C" {

int mpo_gp_kernel_matrix(const double* X, int n, int d, const double* ls, double amp,
                         double diag_add, double* K, int ldk, void* stream) {
    MPO_GUARD_BEGIN
    MPO_CHECK_ARG(X && ls && K, "mpo_gp_kernel_matrix: null pointer");
    MPO_CHECK_ARG(n > 0 && d > 0 && ldk >= n, "mpo_gp_kernel_matrix: bad shape n=%d d=%d ldk=%d", n, d, ldk);
    hipStream_t s = static_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(kernel_matrix_unscaled_kernel, dim3((n + 63) / 64, n), dim3(64), 0, s, X, n, d, ls, amp, diag_add, K, ldk);
    MPO_LAUNCH_CHECK();
    return MPO_OK;
    MPO_GUARD_END
}

int mpo_chol_f64(double* A, int n, int lda, int32_t* info, void* stream) {
    MPO_GUARD_BEGIN
    MPO_CHECK_ARG(A && info, "mpo_chol_f64: null pointer");
    MPO_CHECK_ARG(n > 0 && lda >= n, "mpo_chol_f64: bad shape n=%d lda=%d", n, lda);
    hipLaunchKernelGGL(chol_kernel, dim3(1), dim3(1024), 0, static_cast<hipStream_t>(stream), A, n, lda, info);
    MPO_LAUNCH_CHECK();
    return MPO_OK;
    MPO_GUARD_END
}

int mpo_trsm_f64(const double* L, int n, int lda, double* B, int nrhs, int ldb, int trans, void* stream) {
    MPO_GUARD_BEGIN
    MPO_CHECK_ARG(L && B, "mpo_trsm_f64: null pointer");
    MPO_CHECK_ARG(n > 0 && nrhs > 0 && lda >= n && ldb >= nrhs, "mpo_trsm_f64: bad shape");
    MPO_CHECK_ARG(trans == 0 || trans == 1, "mpo_trsm_f64: trans must be 0 or 1");
    return trsm_launch(L, n, lda, B, nrhs, ldb, trans, static_cast<hipStream_t>(stream));
    MPO_GUARD_END
}

size_t mpo_gp_prepare_ws_bytes(int n, int d) {
    const int dp = pad_dims(d);
    if (n <= 0 || dp < 0) return 0;
    const int np16 = (n + 15) / 16 * 16;
    const int np32 = (n + 31) / 32 * 32;
    mpo::WsCarver c(nullptr);
    c.take<double>((size_t)np32 * dp);     // xs (+ far-away padding rows)
    c.take<double>(dp);                    // ls_pad
    c.take<double>((size_t)n * n);         // L
    c.take<double>((size_t)n * n);         // W
    c.take<double>(np32);                  // alpha (+ zero padding)
    c.take<double>(wfrag_elems(np16));     // wfrag
    c.take<int32_t>(4);                    // info
    return c.used + 256;
}

int mpo_gp_prepare(const double* X, const double* y_norm, int n, int d, const double* ls,
                   double amp, double noise, double y_mean, double y_std,
                   MpoGpModel* model, void* ws, size_t ws_bytes, void* stream) {
    MPO_GUARD_BEGIN
    MPO_CHECK_ARG(X && y_norm && ls && model && ws, "mpo_gp_prepare: null pointer");
    const int dp = pad_dims(d);
    MPO_CHECK_ARG(n > 0 && d > 0, "mpo_gp_prepare: bad shape n=%d d=%d", n, d);
    if (dp < 0) { mpo::set_error("mpo_gp_prepare: d=%d > 32 unsupported", d); return MPO_ENOTSUP; }
    MPO_CHECK_ARG(ws_bytes >= mpo_gp_prepare_ws_bytes(n, d), "mpo_gp_prepare: workspace too small (%zu < %zu)",
                  ws_bytes, mpo_gp_prepare_ws_bytes(n, d));
    const int np16 = (n + 15) / 16 * 16;
    const int np32 = (n + 31) / 32 * 32;
    if (choose_bm(dp, np16) < 0) { mpo::set_error("mpo_gp_prepare: n=%d exceeds the LDS-resident scoring limit", n); return MPO_ENOTSUP; }
    hipStream_t s = static_cast<hipStream_t>(stream);
    mpo::WsCarver c(ws);
    double* xs = c.take<double>((size_t)np32 * dp);
    double* ls_pad = c.take<double>(dp);
    double* L = c.take<double>((size_t)n * n);
    double* W = c.take<double>((size_t)n * n);
    double* alpha = c.take<double>(np32);
    double* wfrag = c.take<double>(wfrag_elems(np16));
    int32_t* info = c.take<int32_t>(4);

    hipLaunchKernelGGL(scale_rows_kernel, dim3((np32 * dp + 255) / 256), dim3(256), 0, s, X, n, np32, d, dp, ls, xs,
                       ls_pad);
    MPO_LAUNCH_CHECK();
    hipLaunchKernelGGL(zero_kernel, dim3((np32 + 255) / 256), dim3(256), 0, s, alpha, np32);
    MPO_LAUNCH_CHECK();
    hipLaunchKernelGGL(kernel_matrix_kernel, dim3((n + 63) / 64, n), dim3(64), 0, s, xs, n, dp, amp,
                       noise + kJitter, L, n);
    MPO_LAUNCH_CHECK();
    hipLaunchKernelGGL(chol_kernel, dim3(1), dim3(1024), 0, s, L, n, n, info);
    MPO_LAUNCH_CHECK();
    hipLaunchKernelGGL(fill_identity_kernel, dim3((n + 63) / 64, n), dim3(64), 0, s, W, n, n);
    MPO_LAUNCH_CHECK();
    int rc = trsm_launch(L, n, n, W, n, n, 0, s);
    if (rc) return rc;
    hipLaunchKernelGGL(copy_kernel, dim3((n + 255) / 256), dim3(256), 0, s, y_norm, alpha, n);
    MPO_LAUNCH_CHECK();
    rc = trsm_launch(L, n, n, alpha, 1, 1, 0, s);
    if (rc) return rc;
    rc = trsm_launch(L, n, n, alpha, 1, 1, 1, s);
    if (rc) return rc;
    const int T = np16 / 16;
    hipLaunchKernelGGL(pack_wfrag_kernel, dim3((4 * T * 64 + 255) / 256, T), dim3(256), 0, s, W, n, n, T, wfrag);
    MPO_LAUNCH_CHECK();

    model->n = n;
    model->d = d;
    model->dp = dp;
    model->np16 = np16;
    model->amp = amp;
    model->y_mean = y_mean;
    model->y_std = y_std;
    model->xs = xs;
    model->ls = ls_pad;
    model->alpha = alpha;
    model->wfrag = wfrag;
    model->L = L;
    model->W = W;
    model->info = info;
    return MPO_OK;
    MPO_GUARD_END
}

size_t mpo_gp_score_ws_bytes(const MpoGpModel* model, int64_t m, int k) {
    if (!model || m <= 0 || k < 0 || k > MPO_TOPK_MAX) return 0;
    if (choose_bm(model->dp, model->np16) < 0) return 0;
    const int64_t nblocks = (m + kWaveTile - 1) / kWaveTile;   // partial lists per 16-candidate tile (upper bound)
    const int kk = std::max(k, 1);
    mpo::WsCarver c(nullptr);
    c.take<long long>((size_t)nblocks * 3 * kk);
    c.take<double>((size_t)nblocks * 3 * kk);
    c.take<long long>((size_t)kMergeGroups * 3 * kk);
    c.take<double>((size_t)kMergeGroups * 3 * kk);
    c.take<long long>(3 * kk);
    c.take<double>(3 * kk);
    return c.used + 256;
}

static int gp_score_impl(const MpoGpModel* model, const double* cand, int64_t m, double y_opt,
                         double xi, double kappa, unsigned flags, int ei_positive, double* mu,
                         double* sd, double* vals, int k, int64_t* topk_idx, double* topk_val,
                         void* ws, size_t ws_bytes, hipStream_t s) {
    MPO_CHECK_ARG(model && cand, "mpo_gp_acq_score: null model/candidates");
    MPO_CHECK_ARG(m > 0, "mpo_gp_acq_score: m must be > 0");
    MPO_CHECK_ARG((flags & ~7u) == 0 && flags != 0, "mpo_gp_acq_score: bad flags %u", flags);
    MPO_CHECK_ARG(k >= 0 && k <= MPO_TOPK_MAX, "mpo_gp_acq_score: k=%d outside [0,%d]", k, MPO_TOPK_MAX);
    MPO_CHECK_ARG(k == 0 || (topk_idx && topk_val), "mpo_gp_acq_score: topk outputs required for k>0");
    MPO_CHECK_ARG(k > 0 || mu || sd || vals, "mpo_gp_acq_score: nothing to compute");
    MPO_CHECK_ARG(ws && ws_bytes >= mpo_gp_score_ws_bytes(model, m, k), "mpo_gp_acq_score: workspace too small");
    const int bm = choose_bm(model->dp, model->np16);
    if (bm < 0) { mpo::set_error("mpo_gp_acq_score: model too large"); return MPO_ENOTSUP; }
    const int64_t nblocks64 = (m + bm - 1) / bm;
    MPO_CHECK_ARG(nblocks64 < (1LL << 31), "mpo_gp_acq_score: too many candidates");
    const int nblocks = (int)nblocks64;
    mpo::WsCarver c(ws);
    const int kk = std::max(k, 1);
    long long* part_idx = c.take<long long>((size_t)nblocks * 3 * kk);
    double* part_val = c.take<double>((size_t)nblocks * 3 * kk);
    long long* mid_idx = c.take<long long>((size_t)kMergeGroups * 3 * kk);
    double* mid_val = c.take<double>((size_t)kMergeGroups * 3 * kk);

    ScoreArgs a;
    a.n = model->n;
    a.np16 = model->np16;
    a.T = model->np16 / 16;
    a.d = model->d;
    a.amp = model->amp;
    a.y_mean = model->y_mean;
    a.y_std = model->y_std;
    a.xs = model->xs;
    a.ls = model->ls;
    a.alpha = model->alpha;
    a.wfrag = model->wfrag;
    a.cand = cand;
    a.m = m;
    a.y_opt = y_opt;
    a.xi = xi;
    a.kappa = kappa;
    a.flags = flags;
    a.ei_positive = ei_positive;
    a.mu = mu;
    a.sd = sd;
    a.vals = vals;
    a.k = k;
    a.part_idx = part_idx;
    a.part_val = part_val;
    const size_t lds = score_lds_bytes(bm, model->dp, model->np16);
    MPO_HIP(launch_score_dp(model->dp, model->d, bm, a, nblocks, lds, s));
    if (k > 0) {
        // stage 1: G groups of ~64 block-lists each; stage 2: one list
        const int chunk = std::max(64, (nblocks + kMergeGroups - 1) / kMergeGroups);
        const int G = (nblocks + chunk - 1) / chunk;
        hipLaunchKernelGGL(topk_merge_kernel, dim3(G, 3), dim3(256), 0, s, part_idx, part_val, nblocks, chunk, k,
                           flags, mid_idx, mid_val, k, 0);
        MPO_LAUNCH_CHECK();
        hipLaunchKernelGGL(topk_merge_kernel, dim3(1, 3), dim3(256), 0, s, mid_idx, mid_val, G, G, k, flags,
                           reinterpret_cast<long long*>(topk_idx), topk_val, k, 1);
        MPO_LAUNCH_CHECK();
    }
    return MPO_OK;
}

int mpo_gp_acq_score(const MpoGpModel* model, const double* cand, int64_t m, double y_opt, double xi,
                     double kappa, unsigned flags, double* mu, double* sd, double* vals, int k,
                     int64_t* topk_idx, double* topk_val, void* ws, size_t ws_bytes, void* stream) {
    MPO_GUARD_BEGIN
    return gp_score_impl(model, cand, m, y_opt, xi, kappa, flags, 0, mu, sd, vals, k, topk_idx, topk_val, ws,
                         ws_bytes, static_cast<hipStream_t>(stream));
    MPO_GUARD_END
}

int mpo_gp_ei_score(const MpoGpModel* model, const double* cand, int64_t m, double y_opt, double xi,
                    double* mu, double* sd, double* ei, int64_t* argmax, void* ws, size_t ws_bytes,
                    void* stream) {
    MPO_GUARD_BEGIN
    MPO_CHECK_ARG(argmax, "mpo_gp_ei_score: null argmax");
    MPO_CHECK_ARG(ws_bytes >= mpo_gp_score_ws_bytes(model, m, 1), "mpo_gp_ei_score: workspace too small");
    // top-1 of -EI lands in the tail of the workspace the score call does not use
    mpo::WsCarver c(ws);
    if (choose_bm(model->dp, model->np16) < 0) { mpo::set_error("mpo_gp_ei_score: model too large"); return MPO_ENOTSUP; }
    const int64_t nblocks = (m + kWaveTile - 1) / kWaveTile;   // the carve of mpo_gp_score_ws_bytes
    c.take<long long>((size_t)nblocks * 3);
    c.take<double>((size_t)nblocks * 3);
    c.take<long long>((size_t)kMergeGroups * 3);
    c.take<double>((size_t)kMergeGroups * 3);
    long long* tidx = c.take<long long>(3);
    double* tval = c.take<double>(3);
    hipStream_t s = static_cast<hipStream_t>(stream);
    int rc = gp_score_impl(model, cand, m, y_opt, xi, 1.96, MPO_ACQ_EI, 1, mu, sd, ei, 1,
                           reinterpret_cast<int64_t*>(tidx), tval, ws, ws_bytes, s);
    if (rc) return rc;
    hipLaunchKernelGGL(argmax_from_topk_kernel, dim3(1), dim3(1), 0, s, tidx, reinterpret_cast<long long*>(argmax));
    MPO_LAUNCH_CHECK();
    return MPO_OK;
    MPO_GUARD_END
}

int mpo_gp_acq_grad(const MpoGpModel* model, const double* x, int batch, const int32_t* acq, double y_opt,
                    double xi, double kappa, double* f, double* g, void* stream) {
    MPO_GUARD_BEGIN
    MPO_CHECK_ARG(model && x && acq && f && g, "mpo_gp_acq_grad: null pointer");
    MPO_CHECK_ARG(batch > 0 && batch <= 65535, "mpo_gp_acq_grad: batch=%d outside [1, 65535]", batch);
    MPO_CHECK_ARG(model->n > 0 && model->d > 0 && model->d <= 32 && model->W, "mpo_gp_acq_grad: model not prepared");
    const size_t lds = (size_t)7 * model->n * sizeof(double);
    if (lds > kMaxLds - 8192) { mpo::set_error("mpo_gp_acq_grad: n=%d too large", model->n); return MPO_ENOTSUP; }
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(acq_grad_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(acq_grad_kernel, dim3(batch), dim3(kGradThreads), lds, static_cast<hipStream_t>(stream),
                       model->n, model->d, model->dp, model->amp, model->y_mean, model->y_std, model->xs, model->ls,
                       model->alpha, model->W, x, acq, y_opt, xi, kappa, f, g);
    MPO_LAUNCH_CHECK();
    return MPO_OK;
    MPO_GUARD_END
}

}  // extern "C"
