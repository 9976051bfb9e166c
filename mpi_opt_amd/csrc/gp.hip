// gp.hip -- fp64 GP posterior + acquisition scoring for gfx950 (MI355X).
//
// Hot path G1-G4 of SURVEY §8a: the skopt "ask" step.  The reference reaches it
// through Coordinator.fit/ask (/root/reference/coordinator.py:63-79, 46-50) ->
// skopt.Optimizer -> GaussianProcessRegressor.predict + gaussian_ei/pi/lcb.
//
// Kernels
//   scale_rows_kernel    xs = X / ls (dims zero-padded to DP)
//   bc_*_kernel          blocked K = L L^T, W = L^-1, alpha (mpo_gp_prepare)
//   chol_kernel          in-place lower Cholesky (one workgroup; mpo_chol_f64)
//   trsm_kernel          L X = B / L^T X = B, one thread per right-hand side (mpo_trsm_f64)
//   pack_wfrag_kernel    L^-1 -> MFMA B-fragment stream (lower triangle only)
//   gp_score_kernel      per 16/32/64-candidate block:
//                          phase 1 (VALU): K*[m][i] = Matern52 into LDS in MFMA
//                                          A-fragment order, mu partials
//                          phase 2 (MFMA): V = K* . L^-T on v_mfma_f64_16x16x4,
//                                          only the lower-triangular k-steps,
//                                          ||V_row||^2 accumulated in registers
//                          phase 3:        sd, mu, -EI/-PI/LCB, block top-k
//   topk_merge_kernel    workgroup top-k lists -> global top-k (lowest index ties)
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
// -k = t ln2 + s, |s| <= ln2/2, with t = round(-k log2 e) from the 1.5*2^52
// rounding constant (no v_rndne), a degree-11 polynomial of e^s fitted at the
// Chebyshev nodes (8.6e-18 relative in exact arithmetic; 13 Taylor terms before),
// 2^t by ldexp from the saturating v_cvt_i32 of t: exp(-k) underflows to exactly
// 0 for every k past ~745 and stays finite for every k < ~1e20 (|xs| far beyond
// what a [0,1]-transformed space with skopt's length-scale bounds produces), so
// no clamp instruction is needed.  Within 2 ulp of exp(-k).
// a*b + c with the constant c read from an SGPR pair.  Written as plain fma the
// compiler keeps loop-invariant coefficients in VGPRs and turns each Horner step
// into v_mov_b64 + v_fmac_f64 (10 extra moves and 20 VGPRs per Matern).
__device__ __forceinline__ double fma_sc(double a, double b, double c) {
    double r;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(c));
    return r;
}

__device__ __forceinline__ double exp_neg(double k) {
    constexpr double kRound = 6755399441055744.0;           // 1.5 * 2^52
    const double t = fma(k, -1.44269504088896340736, kRound) - kRound;
    double x = fma(t, -6.93147180369123816490e-01, -k);
    x = fma(t, -1.90821492927058770002e-10, x);
    double p = 2.511274345242859e-08;
    p = fma_sc(p, x, 2.76326459433635e-07);
    p = fma_sc(p, x, 2.755723242556338e-06);
    p = fma_sc(p, x, 2.4801485486569327e-05);
    p = fma_sc(p, x, 0.00019841269899541455);
    p = fma_sc(p, x, 0.0013888888952271288);
    p = fma_sc(p, x, 0.008333333333315002);
    p = fma_sc(p, x, 0.04166666666648857);
    p = fma_sc(p, x, 0.1666666666666669);
    p = fma_sc(p, x, 0.5000000000000018);
    p = fma(p, x, 1.0);
    p = fma(p, x, 1.0);
    return ldexp(p, (int)t);
}

// sqrt of r2 >= 1e-300 (the distance loops start their sum at 1e-300, so a zero
// distance never reaches v_rsq as 0) by v_rsq_f64, a Goldschmidt step and one
// Newton correction (ocml's sequence without its denormal scaling and 0/inf
// fix-ups).  Within 2 ulp; an ulp of r moves K* by <= 1e-14 relative.
__device__ __forceinline__ double sqrt_pos(double r2) {
    const double y = __builtin_amdgcn_rsq(r2);
    double s = r2 * y, h = 0.5 * y;
    const double e0 = fma(-h, s, 0.5);
    s = fma(s, e0, s);
    h = fma(h, e0, h);
    const double e1 = fma(-s, s, r2);
    return fma(e1, h, s);
}

// first term of every pairwise squared-distance sum (see sqrt_pos)
constexpr double kR2Floor = 1e-300;

// The scoring kernel's Matern WITHOUT the ConstantKernel amplitude:
// (1 + k + k^2/3) exp(-k), k = sqrt(5 r2), k^2/3 = r2 * 5/3.  The kernel folds amp
// into mu (amp * K'.alpha) and into q (amp^2 ||L^-1 K'||^2): one multiply fewer per
// candidate-observation pair -- fp64 VALU and fp64 MFMA work do not overlap on
// gfx950 (scripts/probes/coexec.hip), so every VALU op per pair is kernel time.
__device__ __forceinline__ double matern52_unit(double r2) {
    const double k = sqrt_pos(r2) * kSqrt5;
    return fma(r2, 5.0 / 3.0, 1.0 + k) * exp_neg(k);
}

// scipy.special.ndtr, the kernel of scipy.stats.norm.cdf (skopt's EI / PI): cephes
// ndtr.c's own algorithm -- erf as x T(x^2) / U(x^2) for |x| <= 1, erfc as
// exp(-x^2) P(x) / Q(x) (1 <= x < 8) or R(x) / S(x) (x >= 8), Horner without FMA
// contraction as the host build evaluates it -- instead of the device libm's
// erf / erfc: with the same exp the results are scipy's bits (CPU check of these
// constants: 98.5% of 300k points bit-exact, the rest within 4.4e-16 relative).  The
// scoring pass times the same (1.40 vs 1.40 ms median, same box, profiles/r05/ei_ndtr_ab_ad.log).
namespace cephes {
__constant__ constexpr double kP[9] = {2.46196981473530512524E-10, 5.64189564831068821977E-1, 7.46321056442269912687E0,
                                       4.86371970985681366614E1,   1.96520832956077098242E2, 5.26445194995477358631E2,
                                       9.34528527171957607540E2,   1.02755188689515710272E3, 5.57535335369399327526E2};
__constant__ constexpr double kQ[8] = {1.32281951154744992508E1, 8.67072140885989742329E1, 3.54937778887819891062E2,
                                       9.75708501743205489753E2, 1.82390916687909736289E3, 2.24633760818710981792E3,
                                       1.65666309194161350182E3, 5.57535340817727675546E2};
__constant__ constexpr double kR[6] = {5.64189583547755073984E-1, 1.27536670759978104416E0, 5.01905042251180477414E0,
                                       6.16021097993053585195E0,  7.40974269950448939160E0, 2.97886665372100240670E0};
__constant__ constexpr double kS[6] = {2.26052863220117276590E0, 9.39603524938001434673E0, 1.20489539808096656605E1,
                                       1.70814450747565897222E1, 9.60896809063285878198E0, 3.36907645100081516050E0};
__constant__ constexpr double kT[5] = {9.60497373987051638749E0, 9.00260197203842689217E1, 2.23200534594684319226E3,
                                       7.00332514112805075473E3, 5.55923013010394962768E4};
__constant__ constexpr double kU[5] = {3.35617141647503099647E1, 5.21357949780152679795E2, 4.59432382970980127987E3,
                                       2.26290000613890934246E4, 4.92673942608635921086E4};
constexpr double kMaxLog = 7.09782712893383996843E2;

template <int N>
__device__ __forceinline__ double polevl(double x, const double (&c)[N]) {
#pragma clang fp contract(off)
    double y = c[0];
#pragma unroll
    for (int i = 1; i < N; ++i) y = y * x + c[i];
    return y;
}
template <int N>   // leading coefficient 1
__device__ __forceinline__ double p1evl(double x, const double (&c)[N]) {
#pragma clang fp contract(off)
    double y = x + c[0];
#pragma unroll
    for (int i = 1; i < N; ++i) y = y * x + c[i];
    return y;
}
// erf for |x| <= 1
__device__ __forceinline__ double erf_small(double x) {
#pragma clang fp contract(off)
    const double z = x * x;
    return x * polevl(z, kT) / p1evl(z, kU);
}
// erfc for x >= 1
__device__ __forceinline__ double erfc_large(double x) {
#pragma clang fp contract(off)
    const double z = -x * x;
    if (z < -kMaxLog) return 0.0;
    const double e = exp(z);
    const double y = x < 8.0 ? (e * polevl(x, kP)) / p1evl(x, kQ) : (e * polevl(x, kR)) / p1evl(x, kS);
    return y;
}
}  // namespace cephes

__device__ __forceinline__ double ndtr(double a) {
#pragma clang fp contract(off)
    if (isnan(a)) return a;
    const double x = a * kSqrt1_2;
    const double z = fabs(x);
    if (z < kSqrt1_2) return 0.5 + 0.5 * cephes::erf_small(x);
    // z >= sqrt(1/2); cephes erfc(z) takes its 1 - erf(z) branch below 1
    const double y = 0.5 * (z < 1.0 ? 1.0 - cephes::erf_small(z) : cephes::erfc_large(z));
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

// Rows [n, rows) of xs are zero padding (alpha and the L^-1 fragments are zero
// there): a scoring loop may run over whole 16-observation groups without bounds
// checks; the padding K* values are finite and contribute nothing.

__global__ void scale_rows_kernel(const double* __restrict__ X, int n, int rows, int d, int dp,
                                  const double* __restrict__ ls, double* __restrict__ xs,
                                  double* __restrict__ ls_pad) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < rows * dp) {
        const int i = t / dp, c = t % dp;
        xs[t] = (c < d && i < n) ? X[(size_t)i * d + c] / ls[c] : 0.0;
    }
    if (ls_pad && t < dp) ls_pad[t] = t < d ? ls[t] : 1.0;
}

__global__ void zero_kernel(double* __restrict__ p, int n) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n) p[t] = 0.0;
}

// MFMA form of the candidate-observation distance (gp_score_kernel<.., MD = 1>):
// xb row i = (-2 xs_i, 1, |xs_i|^2, 0 ...), so that [c, |c|^2, 1, 0 ...] . xb_i =
// |c - xs_i|^2 with an absolute rounding error of a few eps (|c|^2 + |xs_i|^2).
// One block; xb[rows * dp] = 1.0 when every |xs_i|^2 <= kDistNorm, else 0.0.
constexpr double kDistNorm = 2.0;
__global__ __launch_bounds__(256) void xb_kernel(const double* __restrict__ xs, int rows, int d, int dp,
                                                 double* __restrict__ xb) {
    __shared__ int bad;
    if (threadIdx.x == 0) bad = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < rows; i += 256) {
        double xx = 0.0;
        for (int c = 0; c < d; ++c) xx = fma(xs[(size_t)i * dp + c], xs[(size_t)i * dp + c], xx);
        for (int c = 0; c < dp; ++c)
            xb[(size_t)i * dp + c] = c < d ? -2.0 * xs[(size_t)i * dp + c] : c == d ? 1.0 : c == d + 1 ? xx : 0.0;
        if (!(xx <= kDistNorm)) atomicOr(&bad, 1);
    }
    __syncthreads();
    if (threadIdx.x == 0) xb[(size_t)rows * dp] = bad ? 0.0 : 1.0;
}

// Self-check of the expanded distance on the model's own observations (r2 = 0 at
// each one's own row and the smallest sd: its worst case): clears the xb flag
// unless both (mu_n, q) rows -- direct and expanded -- agree within 1e-10: q
// relative to sd^2 = amp - q, mu_n relative to its summand scale amp sum |alpha_i|
// (the conditioning of K*.alpha; the parity tests measure mu against the same kind
// of scale).
__global__ __launch_bounds__(256) void xb_check_kernel(const double* __restrict__ mqd, const double* __restrict__ mqm,
                                                       const double* __restrict__ alpha, int n, double amp,
                                                       double* __restrict__ flag) {
    __shared__ int bad;
    __shared__ double red[4];
    if (threadIdx.x == 0) bad = 0;
    double sa = 0.0;
    for (int i = threadIdx.x; i < n; i += 256) sa += fabs(alpha[i]);
    for (int o = 32; o > 0; o >>= 1) sa += __shfl_down(sa, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sa;
    __syncthreads();
    const double mu_scale = amp * (red[0] + red[1] + red[2] + red[3]);
    for (int i = threadIdx.x; i < n; i += 256) {
        const double mud = mqd[2 * i], qd = mqd[2 * i + 1], mum = mqm[2 * i], qm = mqm[2 * i + 1];
        const bool ok = fabs(qm - qd) <= 1e-10 * fmax(amp - qd, 1e-300) && fabs(mum - mud) <= 1e-10 * mu_scale;
        if (!ok) atomicOr(&bad, 1);
    }
    __syncthreads();
    if (threadIdx.x == 0 && bad) flag[0] = 0.0;
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

// B-fragment streams of W^T (W = L^-1 lower), one per scoring wave.
// Column tile jt (16 columns) needs the k-steps ks < 4(jt+1) (rows i <= 16 jt + 15):
// jt+1 groups of 4 k-steps; lane l of k-step ks holds
//   W^T[4 ks + (l>>4)][16 jt + (l&15)] = W[16 jt + (l&15)][4 ks + (l>>4)].
// The T tiles are dealt to the block's 4 waves by LPT on their group counts, and each
// wave's tiles are stored back to back, so a wave reads one contiguous stream across
// its tile boundaries (a software pipeline that never drains), followed by
// kStreamSlack groups of zeros for the prefetch that runs past its end.
// wmeta (int32): wave record w at w*(T+4): [group offset, groups, tiles, jt...];
//                tile_off[jt] at 4*(T+4) + jt (group offset of tile jt's first group).
constexpr int kStreamSlack = 2;   // = the ring depth of the scoring kernel's B pipeline
inline size_t wfrag_elems(int np16) {
    const size_t T = np16 / 16;
    return (T * (T + 1) / 2 + 4 * kStreamSlack) * 256;
}
inline size_t wmeta_elems(int np16) {
    const int T = np16 / 16;
    return (size_t)4 * (T + 4) + T + 4;
}

__global__ void wave_plan_kernel(int T, int32_t* __restrict__ meta) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    int load[4] = {0, 0, 0, 0}, cnt[4] = {0, 0, 0, 0};
    for (int jt = T - 1; jt >= 0; --jt) {       // LPT: costliest tile to the least loaded wave
        int w = 0;
        for (int v = 1; v < 4; ++v)
            if (load[v] < load[w]) w = v;
        meta[w * (T + 4) + 3 + cnt[w]++] = jt;
        load[w] += jt + 1;
    }
    int off = 0;
    for (int w = 0; w < 4; ++w) {
        int32_t* r = meta + w * (T + 4);
        r[0] = off;
        r[1] = load[w];
        r[2] = cnt[w];
        for (int t = cnt[w]; t <= T; ++t) r[3 + t] = 0;
        int g = off;
        for (int t = 0; t < cnt[w]; ++t) {
            meta[4 * (T + 4) + r[3 + t]] = g;
            g += r[3 + t] + 1;
        }
        off += load[w] + kStreamSlack;
    }
}

__global__ void pack_wfrag_kernel(const double* __restrict__ W, int n, int ldw, int T,
                                  const int32_t* __restrict__ meta, double* __restrict__ wfrag) {
    const int jt = blockIdx.y;
    if (jt >= T) return;
    const int nks = 4 * (jt + 1);
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= nks * 64) return;
    const int ks = e >> 6, l = e & 63;
    const int i = 4 * ks + (l >> 4), j = 16 * jt + (l & 15);
    const double v = (i < n && j < n && i <= j) ? W[(size_t)j * ldw + i] : 0.0;
    wfrag[(size_t)meta[4 * (T + 4) + jt] * 256 + e] = v;
}

// ---------------------------------------------------------------------------
constexpr int kBM = 16;   // candidates per scoring workgroup (one 16-row MFMA m-tile)

struct ScoreArgs {
    int n, np16, T, d;
    double amp, y_mean, y_std;
    const double* xs;
    const double* xb;     // MD = 1: augmented observation rows (xb_kernel)
    const double* xb_ok;  // MD = 1: device flag, every |xs_i|^2 <= kDistNorm
    const double* ls;
    const double* alpha;
    const double* wfrag;
    const int32_t* wmeta;
    const double* cand;
    long long m;
    double y_opt, xi, kappa;
    unsigned flags;
    int ei_positive;  // write +EI (mpo_gp_ei_score) instead of -EI into vals
    int dbg;          // MPO_GP_DEBUG phase switches (timing experiments only; results invalid):
                      // bit 0 skips the MFMA phase, bit 1 the Matern arithmetic, bit 2 the top-k,
                      // bit 3 the finish's posterior / acquisition arithmetic
    double* mu;
    double* sd;
    double* vals;
    int k;
    long long* part_idx;  // [nparts][3][k]
    double* part_val;
    double* mq;           // [m][2] raw (mu_n, q) rows (FIN = 0 only: the prepare-time self-check)
};

// One wave, 64 candidates (lane = candidate; invalid lanes contribute nothing): the
// posterior and acquisitions as score_finish_kernel computes them, the requested
// output rows, then the candidates merged into the workgroup's running top-k lists
// (tk_val / tk_idx [3][MPO_TOPK_MAX], sorted, LDS).  A lane takes part only while its
// (value, index) beats the list's k-th entry; each round inserts the group minimum
// among those lanes (lane 0 shifts the list), so at most k rounds run and usually none.
__device__ __attribute__((noinline)) void score_finish_group(const ScoreArgs& a, bool valid, long long gm, double mu_n,
                                                   double q, int lane, double* tk_val, long long* tk_idx) {
    double mu = 0.0, sd = 0.0, vei = 0.0, vpi = 0.0, vlcb = 0.0;
    if (valid && (a.dbg & 8)) {   // timing only: the posterior / acquisition arithmetic skipped
        mu = mu_n;
        sd = q;
    } else if (valid) {
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
        if (a.mu) a.mu[gm] = mu;
        if (a.sd) a.sd[gm] = sd;
        if (a.vals) {
            if (a.flags & MPO_ACQ_EI) a.vals[gm] = a.ei_positive ? -vei : vei;
            if (a.flags & MPO_ACQ_PI) a.vals[a.m + gm] = vpi;
            if (a.flags & MPO_ACQ_LCB) a.vals[2 * a.m + gm] = vlcb;
        }
    }
    if (a.k <= 0 || (a.dbg & 4)) return;
    const double inf = __builtin_huge_val();
    const long long big = 0x7fffffffffffffffLL;
    const int k = a.k;
#pragma unroll
    for (int acq = 0; acq < 3; ++acq) {
        if (!(a.flags & (1u << acq))) continue;
        const double v = valid ? (acq == 0 ? vei : (acq == 1 ? vpi : vlcb)) : inf;
        const long long idx = valid ? gm : big;
        double* lv = tk_val + acq * MPO_TOPK_MAX;
        long long* li = tk_idx + acq * MPO_TOPK_MAX;
        bool cand = valid && lex_less(v, idx, lv[k - 1], li[k - 1]);
        while (__any(cand)) {
            double bv = cand ? v : inf;
            long long bi = cand ? idx : big;
            wave_lex_min(bv, bi);
            if (lane == 0) {
                int pos = k - 1;
                while (pos > 0 && lex_less(bv, bi, lv[pos - 1], li[pos - 1])) {
                    lv[pos] = lv[pos - 1];
                    li[pos] = li[pos - 1];
                    --pos;
                }
                lv[pos] = bv;
                li[pos] = bi;
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // lane 0's list stores before every lane's reads
            cand = cand && idx != bi && lex_less(v, idx, lv[k - 1], li[k - 1]);
        }
    }
}

// One workgroup = 4 waves looping over 16-candidate tiles (kBM) tile = blockIdx.x,
// += gridDim.x (the grid is sized to the resident capacity); the next tile's
// candidate rows are loaded while the current one is scored.
// FIN = 1 (every scoring launch): after its tile loop the workgroup finishes its own
// candidates -- the (mu_n, q) rows it wrote (still largely in this XCD's L2) read
// back 64 per wave with every lane live, the posterior and acquisitions as
// score_finish_group computes them, one running top-k list per wave -- instead of a
// separate finish launch over rows written by workgroups on every XCD.  (An in-loop
// finish was built first: the loop already holds 101 SGPRs and 96 VGPRs at
// occupancy 5, and the finish's invariants spilled it.)  FIN = 0 stops at the rows
// (mpo_gp_prepare's self-check of the expanded form).
template <int DP, int D, int OCC, int MD, int FIN>
__global__ __launch_bounds__(256, OCC) void gp_score_kernel(ScoreArgs a) {
    static_assert(!MD || D + 2 <= DP, "the MFMA distance needs two spare columns");
    constexpr int BM = kBM;
    constexpr int S = 16;            // i-slots per block in phase 1 (4 per wave)
    constexpr int EPT = (BM * DP + 255) / 256;   // candidate elements per thread in phase 0
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int np16 = a.np16;
    double* kc = smem;                          // [np16/4][64]: k-step ks at kc[ks*64]
    double* cs = kc + (size_t)np16 * BM;        // [BM][DP]
    double* red = cs + BM * DP;                 // [S][BM] (mu) then [4][BM] (q)
    int32_t* mls = reinterpret_cast<int32_t*>(red + S * BM);   // the 4 wave records of wmeta

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const long long ntiles = (a.m + BM - 1) / BM;

    for (int e = tid; e < 4 * (a.T + 4); e += 256) mls[e] = a.wmeta[e];

    const bool xb_ok = MD && *a.xb_ok != 0.0;   // read once: the model-level guard of the expanded distance
    // thread tid owns elements tid + 256 u of the [BM][DP] candidate tile
    double raw[EPT], ls_e[EPT];
#pragma unroll
    for (int u = 0; u < EPT; ++u) {
        const int c = (tid + 256 * u) % DP;
        ls_e[u] = c < a.d ? a.ls[c] : 1.0;
    }
#define MPO_LOAD_TILE(TILE)                                                                    \
    _Pragma("unroll") for (int u = 0; u < EPT; ++u) {                                          \
        const int e = tid + 256 * u, r = e / DP, c = e % DP;                                   \
        const long long gm = (TILE) * BM + r;                                                  \
        raw[u] = (e < BM * DP && gm < a.m && c < a.d) ? __builtin_nontemporal_load(a.cand + gm * a.d + c) : 0.0; \
    }
    MPO_LOAD_TILE((long long)blockIdx.x)
    __syncthreads();
    // the finishing wave (mu fold, phase 3, FIN's group finish): the wave whose phase-2
    // B stream (sw = (wave + blockIdx.x) & 3, below) carries the fewest groups
    int fw = 0;
    {
        int lw = 0;
        for (int q = 1; q < 4; ++q)
            if (mls[q * (a.T + 4) + 1] < mls[lw * (a.T + 4) + 1]) lw = q;
        fw = __builtin_amdgcn_readfirstlane((lw - (int)blockIdx.x) & 3);
    }

    // Phase-2 B-fragment stream of this wave (rotated by block so the heaviest one
    // does not always land on the same SIMD).  B fragments arrive through asm loads
    // with explicit vmcnt waits: the compiler's own waitcnt placement drained the
    // ring every iteration (vmcnt(0) before register copies).  The ring lives
    // inside phase 2 only and is drained at its end: a compiler copy of a ring
    // register across a loop back-edge would read it before its load lands (a
    // ring kept in flight across candidate tiles failed parity exactly so).
    const int sw = (wave + (int)blockIdx.x) & 3;
    const int32_t* mw = mls + sw * (a.T + 4);        // LDS: no vmcnt wait at tile ends
    const int G = (a.dbg & 1) ? 0 : __builtin_amdgcn_readfirstlane(mw[1]);
    const double* bs = a.wfrag + (size_t)__builtin_amdgcn_readfirstlane(mw[0]) * 256 + lane;
#define MPO_LD(D, P, OFF) asm volatile("global_load_dwordx2 %0, %1, off offset:" #OFF : "=v"(D) : "v"(P) : "memory")
#define MPO_LD4(B, P) { MPO_LD(B[0], P, 0); MPO_LD(B[1], P, 512); MPO_LD(B[2], P, 1024); MPO_LD(B[3], P, 1536); }

    for (long long tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const long long m0 = tile * BM;

    // ---- phase 0: candidate tile / ls -> LDS; the next tile's rows start loading
#pragma unroll
    for (int u = 0; u < EPT; ++u)
        if (tid + 256 * u < BM * DP) cs[tid + 256 * u] = raw[u] / ls_e[u];
    MPO_LOAD_TILE(tile + gridDim.x)
    __syncthreads();

    // ---- phase 1: K*[row][i] (Matern52) in A-fragment order, mu partials.  xs and
    // alpha hold far-away / zero rows up to np16 + 16: no bounds check on i, and the
    // next observation row is loaded while the current one is evaluated.
    {
        const int row = lane & 15;
        const int slot = wave * 4 + (lane >> 4);
        double c[D];
#pragma unroll
        for (int q = 0; q < D; ++q) c[q] = cs[row * DP + q];
        double mu_acc = 0.0;
        bool md = false;   // this tile on the MFMA distance (every |c|^2 <= kDistNorm)
        if constexpr (MD) {
            double cc = 0.0;
#pragma unroll
            for (int q = 0; q < D; ++q) cc = fma(c[q], c[q], cc);
            md = xb_ok && __all(cc <= kDistNorm);
            if (md && !(a.dbg & 2)) {
                // K*[16 candidates][16 observations] per tile t of this wave: r2 as one
                // augmented dot product on f64 MFMA (A = [c, |c|^2, 1], B = xb), then the
                // Matern per C element.  f64 C/D map: col = lane & 15 (observation),
                // row = (lane >> 4) + 4 r (candidate).
                const int kr = lane >> 4;
                double af[DP / 4];
#pragma unroll
                for (int s = 0; s < DP / 4; ++s) {
                    const int kk = 4 * s + kr;
                    const double v = cs[row * DP + kk];
                    af[s] = kk == D ? cc : kk == D + 1 ? 1.0 : v;
                }
                const int T16 = np16 >> 4;
                const double* xbl = a.xb + (size_t)(lane & 15) * DP + kr;
                double bq[DP / 4];
                double mu4[4] = {0.0, 0.0, 0.0, 0.0};
                for (int t = wave; t < T16; t += 4) {
#pragma unroll
                    for (int s = 0; s < DP / 4; ++s) bq[s] = xbl[(size_t)t * 16 * DP + 4 * s];
                    f64x4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
                    for (int s = 0; s < DP / 4; ++s) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(af[s], bq[s], acc, 0, 0, 0);
                    const int i = t * 16 + (lane & 15);
                    const double al = a.alpha[i];
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const double kv = matern52_unit(fmax(acc[r], kR2Floor));
                        kc[(size_t)(i >> 2) * 64 + kr + 4 * r + (i & 3) * 16] = kv;
                        mu4[r] = fma(kv, al, mu4[r]);
                    }
                }
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    double v = mu4[r];
                    v += __shfl_xor(v, 1);
                    v += __shfl_xor(v, 2);
                    v += __shfl_xor(v, 4);
                    v += __shfl_xor(v, 8);
                    mu4[r] = v;
                }
                // this wave's 4 slots: the sum in slot 0, zeros in 1..3 (the mu fold below
                // sums all 16 slots in order)
                if ((lane & 15) == 0) {
#pragma unroll
                    for (int r = 0; r < 4; ++r)
#pragma unroll
                        for (int q = 0; q < 4; ++q) red[(wave * 4 + q) * BM + kr + 4 * r] = q == 0 ? mu4[r] : 0.0;
                }
            }
        }
        if (md && !(a.dbg & 2)) {
        } else if (a.dbg & 2) {
            for (int i = slot; i < np16; i += S) kc[(size_t)(i >> 2) * 64 + row + (i & 3) * 16] = c[0];
        } else {
            // one observation row: r2, Matern, mu partial, K* into LDS
#define MPO_EI_PAIR(XC, AC, I)                                                                     \
            {                                                                                      \
                double r2 = kR2Floor;                                                              \
                _Pragma("unroll") for (int q = 0; q < D; ++q) {                                    \
                    const double t = c[q] - XC[q];                                                 \
                    r2 = fma(t, t, r2);                                                            \
                }                                                                                  \
                const double kv = matern52_unit(r2);   /* amp folded into mu and q below */        \
                mu_acc = fma(kv, AC, mu_acc);                                                      \
                kc[(size_t)((I) >> 2) * 64 + row + ((I) & 3) * 16] = kv;                           \
            }
            for (int i = slot; i < np16; i += S) {
                const double* xr = a.xs + (size_t)i * DP;
                MPO_EI_PAIR(xr, a.alpha[i], i)
            }
#undef MPO_EI_PAIR
        }
        if (!md || (a.dbg & 2)) red[slot * BM + row] = mu_acc;
    }
    __syncthreads();
    double mu_n = 0.0;
    if (wave == fw && lane < BM) {
#pragma unroll
        for (int s = 0; s < S; ++s) mu_n += red[s * BM + lane];
        mu_n *= a.amp;
    }
    __syncthreads();  // red is reused for the q partials below

    // ---- phase 2: V = K* L^-T on f64 MFMA, lower-triangular k-steps only.  The
    // wave walks its B-fragment stream (wave_plan_kernel) two 4-k-step groups ahead
    // (loading the ring's first groups before the mu barriers instead measured the same).
    {
        double b0[4], b1[4];
        MPO_LD4(b0, bs);
        MPO_LD4(b1, bs + 256);
        const double* bp = bs + 512;
        const double* kl = kc + lane;
        double sq[4] = {0.0, 0.0, 0.0, 0.0};
        f64x4 acc0 = {0.0, 0.0, 0.0, 0.0}, acc1 = {0.0, 0.0, 0.0, 0.0};
        int t = 0, kg = 0, tlen = __builtin_amdgcn_readfirstlane(mw[3] + 1);
        // one group: 4 MFMAs on two accumulation chains, then the ring slot is
        // refilled with the group two ahead; at a column tile's last group
        // ||V_row||^2 takes the tile's columns
#define MPO_EI_GROUP(B)                                                                            \
        {                                                                                          \
            asm volatile("s_waitcnt vmcnt(4)" : "+v"(B[0]), "+v"(B[1]), "+v"(B[2]), "+v"(B[3])); \
            const double* ap = kl + kg * 256;                                                      \
            acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(ap[0], B[0], acc0, 0, 0, 0);              \
            acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(ap[64], B[1], acc1, 0, 0, 0);             \
            acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(ap[128], B[2], acc0, 0, 0, 0);            \
            acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(ap[192], B[3], acc1, 0, 0, 0);            \
            MPO_LD4(B, bp);                                                                        \
            bp += 256;                                                                             \
            if (++kg == tlen) {                                                                    \
                _Pragma("unroll") for (int r = 0; r < 4; ++r) {                                    \
                    const double v = acc0[r] + acc1[r];                                            \
                    sq[r] = fma(v, v, sq[r]);                                                      \
                }                                                                                  \
                acc0 = f64x4{0.0, 0.0, 0.0, 0.0};                                                  \
                acc1 = f64x4{0.0, 0.0, 0.0, 0.0};                                                  \
                kg = 0;                                                                            \
                tlen = __builtin_amdgcn_readfirstlane(mw[3 + (++t)] + 1);                          \
            }                                                                                      \
        }
        for (int g = 0; g < G; g += 2) {
            MPO_EI_GROUP(b0)
            if (g + 1 >= G) break;
            MPO_EI_GROUP(b1)
        }
        asm volatile("s_waitcnt vmcnt(0)" : "+v"(b0[0]), "+v"(b0[1]), "+v"(b0[2]), "+v"(b0[3]), "+v"(b1[0]),
                     "+v"(b1[1]), "+v"(b1[2]), "+v"(b1[3]));
#undef MPO_EI_GROUP
        // f64 C/D map: col = lane & 15, row = (lane >> 4) + 4 r.  Sum the columns.
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            double v = sq[r];
            v += __shfl_xor(v, 1);
            v += __shfl_xor(v, 2);
            v += __shfl_xor(v, 4);
            v += __shfl_xor(v, 8);
            if ((lane & 15) == 0) red[wave * BM + (lane >> 4) + 4 * r] = v;
        }
    }
    __syncthreads();

    // ---- phase 3: (mu_n, q) rows out (wave fw; the other waves go on to the next
    // tile's phase 0 and meet wave fw at its barrier, after which red may be rewritten)
    if (wave == fw && lane < BM && m0 + lane < a.m) {
        const double q = (red[0 * BM + lane] + red[1 * BM + lane] + red[2 * BM + lane] + red[3 * BM + lane]) *
                         (a.amp * a.amp);
        *reinterpret_cast<double2*>(a.mq + 2 * (m0 + lane)) = double2{mu_n, q};
    }
    }  // tile loop
    if constexpr (FIN) {
        // ---- finish: this workgroup's own (mu_n, q) rows (written above, mostly still
        // in this XCD's L2), 64 candidates per wave at a time with every lane live;
        // one running top-k list per wave in the (now free) K* LDS region
        __syncthreads();   // the rows of wave fw (global writes, workgroup-scope visibility)
        // the finish reads its arguments through a pointer to the kernarg segment: the
        // out-of-line score_finish_group given `a` itself would copy the by-value
        // struct to the stack (and the scoring variants must stay scratch-free, see
        // launch_score); the asm keeps the loads out of the tile loop
        const ScoreArgs* ap = (const ScoreArgs*)__builtin_amdgcn_kernarg_segment_ptr();
        asm volatile("" : "+s"(ap));
        const ScoreArgs& f = *ap;
        double* tk_val = kc + wave * 3 * MPO_TOPK_MAX;
        long long* tk_idx = reinterpret_cast<long long*>(kc + 4 * 3 * MPO_TOPK_MAX) + wave * 3 * MPO_TOPK_MAX;
        if (lane < 3 * MPO_TOPK_MAX) {
            tk_val[lane] = __builtin_huge_val();
            tk_idx[lane] = 0x7fffffffffffffffLL;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const long long ntl = ((f.m + BM - 1) / BM - blockIdx.x + gridDim.x - 1) / gridDim.x;   // this workgroup's tiles
        for (long long c0 = (long long)wave * 64; c0 < ntl * BM; c0 += 256) {
            const long long cl = c0 + lane;
            const long long gm = (blockIdx.x + (cl >> 4) * (long long)gridDim.x) * BM + (cl & 15);
            const bool valid = cl < ntl * BM && gm < f.m;
            double2 v = {0.0, 0.0};
            if (valid) v = *reinterpret_cast<const double2*>(f.mq + 2 * gm);
            score_finish_group(f, valid, gm, v.x, v.y, lane, tk_val, tk_idx);
        }
        if (f.k > 0 && lane < 3 * f.k) {
            const int acq = lane / f.k, r = lane - acq * f.k;
            const size_t part = (size_t)blockIdx.x * 4 + wave;
            f.part_val[(part * 3 + acq) * f.k + r] = tk_val[acq * MPO_TOPK_MAX + r];
            f.part_idx[(part * 3 + acq) * f.k + r] = tk_idx[acq * MPO_TOPK_MAX + r];
        }
    }
#undef MPO_LD4
#undef MPO_LD
#undef MPO_LOAD_TILE
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
// Scoring grid bound: the resident capacity is <= 8 workgroups of 4 waves per CU
// (32 waves), 256 CUs on MI355X; workspace for top-k lists is sized from this.
constexpr int kScoreGridCap = 8 * 256;

size_t score_lds_bytes(int dp, int np16) {
    const int T = np16 / 16;
    // kc (after the tile loop: FIN's per-wave top-k lists, 4 x 3 x MPO_TOPK_MAX x 16 B <= np16 x kBM x 8 B),
    // cs, red | wave records
    return ((size_t)np16 * kBM + (size_t)kBM * dp + 16 * kBM) * sizeof(double) + (size_t)4 * (T + 4) * sizeof(int32_t);
}

bool score_fits(int dp, int np16) { return score_lds_bytes(dp, np16) <= kMaxLds; }

// grid = the device's resident capacity for this variant (tiles are looped over);
// *grid_out receives it (FIN: one top-k list per workgroup)
template <int DP, int D, int OCC, int MD, int FIN>
hipError_t launch_score(const ScoreArgs& a, int ntiles, size_t lds, hipStream_t s, int* grid_out) {
    auto kern = gp_score_kernel<DP, D, OCC, MD, FIN>;
    // The B ring's asm loads are invisible to the compiler: a spill of a ring
    // register would store it before its load lands.  A variant whose register
    // cap forces spills is refused instead of run.
    hipFuncAttributes fa;
    if (hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(kern)) != hipSuccess || fa.localSizeBytes != 0)
        return hipErrorInvalidDeviceFunction;
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                        (int)lds);
    int dev = 0, cus = 0, per_cu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(kern), 256, lds);
    int grid = std::max(1, std::min(std::min(ntiles, kScoreGridCap), std::max(1, per_cu) * std::max(1, cus)));
    if (grid_out) *grid_out = grid;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, s, a);
    return hipGetLastError();
}

template <int DP, int D, int OCC, int MD, int FIN>
bool spill_free() {
    static int ok = -1;
    if (ok < 0) {
        hipFuncAttributes fa;
        ok = hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(gp_score_kernel<DP, D, OCC, MD, FIN>)) ==
                 hipSuccess &&
             fa.localSizeBytes == 0;
    }
    return ok == 1;
}

// occupancy hint (min waves per SIMD -> VGPR cap): the highest spill-free one;
// MPO_GP_OCC (2, 4, 5, 6) forces one for experiments
template <int DP, int D, int MD, int FIN>
hipError_t launch_score_occ_md(const ScoreArgs& a, int nblocks, size_t lds, hipStream_t s, int* grid_out) {
    const char* e = getenv("MPO_GP_OCC");
    int occ = e ? atoi(e) : 0;
    if (occ != 2 && occ != 4 && occ != 5 && occ != 6)
        occ = spill_free<DP, D, 6, MD, FIN>()   ? 6
              : spill_free<DP, D, 5, MD, FIN>() ? 5
              : spill_free<DP, D, 4, MD, FIN>() ? 4
                                                : 2;
    switch (occ) {
        case 6: return launch_score<DP, D, 6, MD, FIN>(a, nblocks, lds, s, grid_out);
        case 5: return launch_score<DP, D, 5, MD, FIN>(a, nblocks, lds, s, grid_out);
        case 4: return launch_score<DP, D, 4, MD, FIN>(a, nblocks, lds, s, grid_out);
        default: return launch_score<DP, D, 2, MD, FIN>(a, nblocks, lds, s, grid_out);
    }
}

// MD = 1 (the MFMA distance) when the model carries xb (d + 2 <= dp; the kernel
// reads the self-check's device flag); MPO_GP_DIST=0 forces the direct form.
// fin = false: raw (mu_n, q) rows only.
template <int DP, int D>
hipError_t launch_score_occ(const ScoreArgs& a, int nblocks, size_t lds, hipStream_t s, bool fin, int* grid_out) {
    if constexpr (D + 2 <= DP) {
        const char* e = getenv("MPO_GP_DIST");
        if (a.xb && a.xb_ok && !(e && e[0] == '0'))
            return fin ? launch_score_occ_md<DP, D, 1, 1>(a, nblocks, lds, s, grid_out)
                       : launch_score_occ_md<DP, D, 1, 0>(a, nblocks, lds, s, grid_out);
    }
    return fin ? launch_score_occ_md<DP, D, 0, 1>(a, nblocks, lds, s, grid_out)
               : launch_score_occ_md<DP, D, 0, 0>(a, nblocks, lds, s, grid_out);
}

// (padded row width DP, distance dims D): d = 5 and d = 10 (the reference's mnist
// space and the BASELINE config) get exact-width distance loops
hipError_t launch_score_dp(int dp, int d, const ScoreArgs& a, int nblocks, size_t lds, hipStream_t s, bool fin,
                           int* grid_out = nullptr) {
    switch (dp) {
        case 4: return launch_score_occ<4, 4>(a, nblocks, lds, s, fin, grid_out);
        case 8: return d == 5 ? launch_score_occ<8, 5>(a, nblocks, lds, s, fin, grid_out)
                              : launch_score_occ<8, 8>(a, nblocks, lds, s, fin, grid_out);
        case 12: return d == 10 ? launch_score_occ<12, 10>(a, nblocks, lds, s, fin, grid_out)
                                : launch_score_occ<12, 12>(a, nblocks, lds, s, fin, grid_out);
        case 16: return launch_score_occ<16, 16>(a, nblocks, lds, s, fin, grid_out);
        case 32: return launch_score_occ<32, 32>(a, nblocks, lds, s, fin, grid_out);
    }
    return hipErrorInvalidValue;
}


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
// Blocked factorisation for mpo_gp_prepare: K = L L^T and W = L^-1 over 32-wide
// blocks on the padded np x np matrix (np = n rounded up to 32, identity on the
// padding, so padded rows never couple to K).  The one-workgroup right-looking
// chol_kernel + one-thread-per-column trsm_kernel took ~27 ms at n = 500 (a cl_min
// batch pays one prepare per lie); here the sequential depth is one 32x32 block
// per step and everything else is MFMA work over many workgroups:
//   per block k:  bc_diag_kernel   (one wave) L_kk = chol(A_kk) in registers and
//                                  D_k = L_kk^-1 (row-wise forward substitution)
//                 bc_panel_kernel  L_ik = A_ik D_k^T for the 16-row tiles below
//                 bc_update_kernel A_IJ -= L_Ik L_Jk^T over the trailing lower tiles
//   per block row I of W:  bc_winv_kernel  W_II = D_I,
//                                          W_IJ = -D_I sum_{K=J}^{I-1} L_IK W_KJ
//   alpha = K^-1 y = W^T (W y)   (bc_wy_kernel, bc_wtv_kernel)
// All sums run in a fixed order: the results do not depend on the launch geometry.
constexpr int kBc = 32;
__host__ __device__ inline int bc_np(int n) { return (n + kBc - 1) / kBc * kBc; }

// A (padded, row-major [np][np]): the lower triangle and the full diagonal 32x32 blocks
__global__ void bc_kmat_kernel(const double* __restrict__ xs, int n, int dp, double amp, double diag_add,
                               double* __restrict__ A, int np) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    const int i = blockIdx.y;
    if (j >= np || j > (i | (kBc - 1))) return;
    double v;
    if (i >= n || j >= n) {
        v = i == j ? 1.0 : 0.0;
    } else {
        double r2 = 0.0;
        for (int c = 0; c < dp; ++c) {
            const double t = xs[(size_t)i * dp + c] - xs[(size_t)j * dp + c];
            r2 += t * t;
        }
        v = matern52(sqrt(r2), amp);
        if (i == j) v += diag_add;
    }
    A[(size_t)i * np + j] = v;
}

// One wave: lane l (and l + 32, mirrored) holds row l of the diagonal block.  Column
// c of the factor is broadcast through the LDS at each step; a non-positive or
// non-finite pivot records info = first failing column + 1 (sklearn's LinAlgError).
__global__ __launch_bounds__(64) void bc_diag_kernel(double* __restrict__ A, int np, int k,
                                                     double* __restrict__ Dinv, double* __restrict__ Wp,
                                                     int32_t* __restrict__ info) {
    __shared__ double col[kBc];
    __shared__ double qrow[kBc];
    const int lane = threadIdx.x, l = lane & (kBc - 1);
    const int k0 = k * kBc;
    double* Akk = A + (size_t)k0 * np + k0;
    double r[kBc];
#pragma unroll
    for (int j = 0; j < kBc; ++j) r[j] = j <= l ? Akk[(size_t)l * np + j] : 0.0;
    int bad = 0;
#pragma unroll
    for (int c = 0; c < kBc; ++c) {
        if (lane < kBc) col[l] = r[c];
        __syncthreads();
        const double d = col[c];
        if (!(d > 0.0) || !isfinite(d)) bad = bad ? bad : c + 1;
        const double lcc = sqrt(d);
        const double inv = 1.0 / lcc;
        if (l > c) r[c] *= inv;
        if (l == c) r[c] = lcc;
#pragma unroll
        for (int j = c + 1; j < kBc; ++j)
            if (j <= l) r[j] = fma(-r[c], col[j] * inv, r[j]);
        __syncthreads();
    }
    // D = L_kk^-1: row c = (e_c - sum_{m<c} L[c][m] D[m]) / L[c][c]; lane l keeps its
    // partial row p and finishes it at step c = l
    double p[kBc];
#pragma unroll
    for (int j = 0; j < kBc; ++j) p[j] = j == l ? 1.0 : 0.0;
#pragma unroll
    for (int c = 0; c < kBc; ++c) {
        if (lane == c) {
            const double inv = 1.0 / r[c];
#pragma unroll
            for (int j = 0; j <= c; ++j) {
                p[j] *= inv;
                qrow[j] = p[j];
            }
        }
        __syncthreads();
        if (l > c) {
#pragma unroll
            for (int j = 0; j <= c; ++j) p[j] = fma(-r[c], qrow[j], p[j]);
        }
        __syncthreads();
    }
    if (lane < kBc) {
#pragma unroll
        for (int j = 0; j < kBc; ++j) {
            if (j <= l) Akk[(size_t)l * np + j] = r[j];
            Dinv[(size_t)k * kBc * kBc + l * kBc + j] = j <= l ? p[j] : 0.0;
            Wp[(size_t)(k0 + l) * np + k0 + j] = j <= l ? p[j] : 0.0;
        }
    }
    if (lane == 0 && bad && info[0] == 0) info[0] = k0 + bad;
}

// L_ik = A_ik D_k^T for the 16-row tiles below block k, one tile per wave
// (two 16-column MFMA outputs, K = 32).  f64 16x16x4 operands: A[m = lane & 15][kk =
// lane >> 4], B[kk = lane >> 4][n = lane & 15]; C/D: col = lane & 15, row = (lane >> 4) + 4 q.
__global__ __launch_bounds__(256) void bc_panel_kernel(double* __restrict__ A, int np, int k,
                                                       const double* __restrict__ Dinv) {
    const int lane = threadIdx.x & 63;
    const int R = (k + 1) * 2 + blockIdx.x * 4 + (threadIdx.x >> 6);
    if (R >= np / 16) return;
    const int k0 = k * kBc;
    const double* D = Dinv + (size_t)k * kBc * kBc;
    f64x4 acc0 = {0.0, 0.0, 0.0, 0.0}, acc1 = {0.0, 0.0, 0.0, 0.0};
    double a[8];
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) a[ks] = A[(size_t)(16 * R + (lane & 15)) * np + k0 + 4 * ks + (lane >> 4)];
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
        const int kk = 4 * ks + (lane >> 4);
        acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a[ks], D[(lane & 15) * kBc + kk], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a[ks], D[(16 + (lane & 15)) * kBc + kk], acc1, 0, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        double* row = A + (size_t)(16 * R + (lane >> 4) + 4 * q) * np + k0;
        row[lane & 15] = acc0[q];
        row[16 + (lane & 15)] = acc1[q];
    }
}

// A_IJ -= L_Ik L_Jk^T over the lower 16x16 tiles of the trailing matrix (I >= J past
// block k), one tile per wave at a time, K = 32 (8 MFMAs)
__global__ __launch_bounds__(256) void bc_update_kernel(double* __restrict__ A, int np, int k) {
    const int lane = threadIdx.x & 63;
    const int t0 = (k + 1) * 2;                 // first trailing 16-tile
    const int T = np / 16 - t0;
    const int ntl = T * (T + 1) / 2;
    const int k0 = k * kBc;
    const int gw = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * 4 + (threadIdx.x >> 6)));
    const int nw = gridDim.x * 4;
    for (int t = gw; t < ntl; t += nw) {
        int I = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
        while (I * (I + 1) / 2 > t) --I;
        while ((I + 1) * (I + 2) / 2 <= t) ++I;
        const int J = t - I * (I + 1) / 2;
        const int gi = 16 * (t0 + I), gj = 16 * (t0 + J);
        f64x4 acc;
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[q] = A[(size_t)(gi + (lane >> 4) + 4 * q) * np + gj + (lane & 15)];
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) {
            const int kk = k0 + 4 * ks + (lane >> 4);
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(-A[(size_t)(gi + (lane & 15)) * np + kk],
                                                       A[(size_t)(gj + (lane & 15)) * np + kk], acc, 0, 0, 0);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) A[(size_t)(gi + (lane >> 4) + 4 * q) * np + gj + (lane & 15)] = acc[q];
    }
}

// Block row I of W = L^-1, block column J = blockIdx.x < I: wave w computes the
// 16x16 tile (a, b) = (w >> 1, w & 1) of S = sum_{K=J}^{I-1} L_IK W_KJ into the LDS,
// then W_IJ = -D_I S.
__global__ __launch_bounds__(256) void bc_winv_kernel(const double* __restrict__ L, double* __restrict__ Wp, int np,
                                                      int I, const double* __restrict__ Dinv) {
    __shared__ double S[kBc][kBc + 1];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int a = w >> 1, b = w & 1;
    const int J = blockIdx.x;
    const int I0 = I * kBc, J0 = J * kBc;
    f64x4 acc = {0.0, 0.0, 0.0, 0.0};
    for (int K = J; K < I; ++K) {
        const int K0 = K * kBc;
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) {
            const int kk = 4 * ks + (lane >> 4);
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(L[(size_t)(I0 + 16 * a + (lane & 15)) * np + K0 + kk],
                                                       Wp[(size_t)(K0 + kk) * np + J0 + 16 * b + (lane & 15)], acc,
                                                       0, 0, 0);
        }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) S[16 * a + (lane >> 4) + 4 * q][16 * b + (lane & 15)] = acc[q];
    __syncthreads();
    const double* D = Dinv + (size_t)I * kBc * kBc;
    f64x4 o = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
        const int kk = 4 * ks + (lane >> 4);
        o = __builtin_amdgcn_mfma_f64_16x16x4f64(D[(16 * a + (lane & 15)) * kBc + kk], S[kk][16 * b + (lane & 15)], o,
                                                 0, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) Wp[(size_t)(I0 + 16 * a + (lane >> 4) + 4 * q) * np + J0 + 16 * b + (lane & 15)] = -o[q];
}

// v = W y (one wave per row, fixed butterfly), then alpha = W^T v (one thread per column)
__global__ __launch_bounds__(256) void bc_wy_kernel(const double* __restrict__ Wp, int np, int n,
                                                    const double* __restrict__ y, double* __restrict__ v) {
    const int lane = threadIdx.x & 63;
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= np) return;
    double s = 0.0;
    for (int j = lane; j <= i && j < n; j += 64) s = fma(Wp[(size_t)i * np + j], y[j], s);
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off);
    if (lane == 0) v[i] = s;
}

__global__ void bc_wtv_kernel(const double* __restrict__ Wp, int np, int n, const double* __restrict__ v,
                              double* __restrict__ alpha) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    double s = 0.0;
    for (int i = j; i < np; ++i) s = fma(Wp[(size_t)i * np + j], v[i], s);
    alpha[j] = s;
}

// padded factors -> the model's [n][n] L and W (lower triangles, zeros above)
__global__ void bc_copy_out_kernel(const double* __restrict__ A, const double* __restrict__ Wp, int np, int n,
                                   double* __restrict__ L, double* __restrict__ W) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    const int i = blockIdx.y;
    if (j >= n) return;
    L[(size_t)i * n + j] = j <= i ? A[(size_t)i * np + j] : 0.0;
    W[(size_t)i * n + j] = j <= i ? Wp[(size_t)i * np + j] : 0.0;
}

// The launch sequence of the blocked factorisation (+ alpha) on stream s.
hipError_t blocked_factor(const double* xs, int n, int dp, double amp, double diag_add, const double* y_norm,
                          double* A, double* Wp, double* Dinv, double* v, double* L, double* W, double* alpha,
                          int32_t* info, hipStream_t s) {
    const int np = bc_np(n), nbk = np / kBc;
    (void)hipMemsetAsync(info, 0, sizeof(int32_t), s);
    (void)hipMemsetAsync(Wp, 0, (size_t)np * np * sizeof(double), s);
    hipLaunchKernelGGL(bc_kmat_kernel, dim3((np + 63) / 64, np), dim3(64), 0, s, xs, n, dp, amp, diag_add, A, np);
    for (int k = 0; k < nbk; ++k) {
        hipLaunchKernelGGL(bc_diag_kernel, dim3(1), dim3(64), 0, s, A, np, k, Dinv, Wp, info);
        const int below = np / 16 - (k + 1) * 2;
        if (below <= 0) continue;
        hipLaunchKernelGGL(bc_panel_kernel, dim3((below + 3) / 4), dim3(256), 0, s, A, np, k, Dinv);
        const int ntl = below * (below + 1) / 2;
        hipLaunchKernelGGL(bc_update_kernel, dim3(std::max(1, std::min(1024, (ntl + 3) / 4))), dim3(256), 0, s,
                           A, np, k);
    }
    for (int I = 1; I < nbk; ++I)
        hipLaunchKernelGGL(bc_winv_kernel, dim3(I), dim3(256), 0, s, A, Wp, np, I, Dinv);
    hipLaunchKernelGGL(bc_wy_kernel, dim3((np + 3) / 4), dim3(256), 0, s, Wp, np, n, y_norm, v);
    hipLaunchKernelGGL(bc_wtv_kernel, dim3((n + 255) / 256), dim3(256), 0, s, Wp, np, n, v, alpha);
    hipLaunchKernelGGL(bc_copy_out_kernel, dim3((n + 63) / 64, n), dim3(64), 0, s, A, Wp, np, n, L, W);
    return hipGetLastError();
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
// LDS: k*, c (n each), v = W k* (n), one per-wave partial of W^T v per wave (NW n).
// NW = 16 waves per point while (3 + NW) n doubles fit the LDS (n <= ~1000; the
// 4-wave form past it): the two triangular mat-vecs are the kernel's serial work,
// 16 waves cut them 4x (n = 512: 214 -> see DESIGN §3.1b round trip per launch).
template <int NW>
__global__ __launch_bounds__(NW * 64) void acq_grad_kernel(
        int n, int d, int dp, double amp, double y_mean, double y_std, const double* __restrict__ xs,
        const double* __restrict__ ls, const double* __restrict__ alpha, const double* __restrict__ W,
        const double* __restrict__ x, const int32_t* __restrict__ acq, double y_opt, double xi, double kappa,
        double* __restrict__ f, double* __restrict__ g) {
    extern __shared__ double sm[];
    double* kk = sm;              // [n]
    double* cc = kk + n;          // [n]
    double* vv = cc + n;          // [n]
    double* up = vv + n;          // [NW][n]
    __shared__ double xp[32];     // x / ls
    constexpr int kGradThreads = NW * 64, kGroups = kGradThreads / 32;
    __shared__ double red[kGradThreads];
    __shared__ double ga[kGroups][32], gu[kGroups][32];
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
    for (int i = tid; i < NW * n; i += kGradThreads) up[i] = 0.0;
    __syncthreads();

    // v = W k* (rows per wave, lanes across the row), q = ||v||^2
    double q_part = 0.0;
    for (int r = wave; r < n; r += NW) {
        double s = 0.0;
        for (int c = lane; c <= r; c += 64) s = fma(W[(size_t)r * n + c], kk[c], s);
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off);
        if (lane == 0) vv[r] = s;
        q_part = fma(s, s, q_part);     // identical in every lane: count lane 0 only
    }
    if (lane != 0) q_part = 0.0;
    __syncthreads();

    // u = W^T v: wave w accumulates rows r = w (mod NW) into its own partial
    double* uw = up + (size_t)wave * n;
    for (int r = wave; r < n; r += NW) {
        const double vr = vv[r];
        for (int c = lane; c <= r; c += 64) uw[c] = fma(W[(size_t)r * n + c], vr, uw[c]);
    }
    __syncthreads();
    for (int i = tid; i < n; i += kGradThreads) {
        double u = up[i];
#pragma unroll
        for (int w = 1; w < NW; ++w) u += up[(size_t)w * n + i];
        up[i] = u;
    }

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

    // dk^T alpha and dk^T u per dimension: thread (grp, j) sums observations grp (mod kGroups)
    {
        const int j = tid & 31, grp = tid >> 5;
        double sa = 0.0, su = 0.0;
        if (j < d) {
            for (int i = grp; i < n; i += kGroups) {
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
        for (int grp = 0; grp < kGroups; ++grp) {
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

// Scoring workspace: per-wave partial top-k lists, the stage-1 merge lists, a
// 3-entry tail (mpo_gp_ei_score's top-1) and the (mu_n, q) rows.
struct ScoreWs {
    long long* part_idx;
    double* part_val;
    long long* mid_idx;
    double* mid_val;
    long long* tail_idx;
    double* tail_val;
    double* mq;
};

// top-k lists: 4 per workgroup (one per wave); a workgroup has at least one tile
// and the grid never exceeds kScoreGridCap (tiles are looped over)
inline int64_t score_nparts(int64_t m) { return 4 * std::min<int64_t>((m + kBM - 1) / kBM, kScoreGridCap); }

inline ScoreWs carve_score_ws(void* ws, int64_t m, int k, size_t* used) {
    const int64_t nparts = score_nparts(m);
    const int kk = std::max(k, 1);
    mpo::WsCarver c(ws);
    ScoreWs w;
    w.part_idx = c.take<long long>((size_t)nparts * 3 * kk);
    w.part_val = c.take<double>((size_t)nparts * 3 * kk);
    w.mid_idx = c.take<long long>((size_t)kMergeGroups * 3 * kk);
    w.mid_val = c.take<double>((size_t)kMergeGroups * 3 * kk);
    w.tail_idx = c.take<long long>(3 * kk);
    w.tail_val = c.take<double>(3 * kk);
    w.mq = c.take<double>((size_t)m * 2);
    if (used) *used = c.used;
    return w;
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
    const int xrows = np16 + 32;           // the scoring kernel reads one 16-row step past np16
    mpo::WsCarver c(nullptr);
    c.take<double>((size_t)xrows * dp);    // xs (+ far-away padding rows)
    c.take<double>(dp);                    // ls_pad
    c.take<double>((size_t)n * n);         // L
    c.take<double>((size_t)n * n);         // W
    c.take<double>(xrows);                 // alpha (+ zero padding)
    c.take<double>(wfrag_elems(np16));     // wfrag
    c.take<int32_t>(4);                    // info
    c.take<int32_t>(wmeta_elems(np16));    // wmeta
    c.take<double>((size_t)xrows * dp + 8);   // xb + its guard flag
    c.take<double>(4 * (size_t)n);            // xb self-check (mu_n, q) rows, direct and expanded
    const size_t np = bc_np(n);
    c.take<double>(np * np);                  // blocked factorisation: padded A -> L
    c.take<double>(np * np);                  //                        padded W
    c.take<double>(np * kBc);                 //                        diagonal-block inverses
    c.take<double>(np);                       //                        W y
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
    const int xrows = np16 + 32;
    if (!score_fits(dp, np16)) { mpo::set_error("mpo_gp_prepare: n=%d exceeds the LDS-resident scoring limit", n); return MPO_ENOTSUP; }
    hipStream_t s = static_cast<hipStream_t>(stream);
    mpo::WsCarver c(ws);
    double* xs = c.take<double>((size_t)xrows * dp);
    double* ls_pad = c.take<double>(dp);
    double* L = c.take<double>((size_t)n * n);
    double* W = c.take<double>((size_t)n * n);
    double* alpha = c.take<double>(xrows);
    double* wfrag = c.take<double>(wfrag_elems(np16));
    int32_t* info = c.take<int32_t>(4);
    int32_t* wmeta = c.take<int32_t>(wmeta_elems(np16));
    double* xb = c.take<double>((size_t)xrows * dp + 8);
    double* mqc = c.take<double>(4 * (size_t)n);
    const size_t npb = bc_np(n);
    double* Ab = c.take<double>(npb * npb);
    double* Wb = c.take<double>(npb * npb);
    double* Db = c.take<double>(npb * kBc);
    double* vb = c.take<double>(npb);

    hipLaunchKernelGGL(scale_rows_kernel, dim3((xrows * dp + 255) / 256), dim3(256), 0, s, X, n, xrows, d, dp, ls, xs,
                       ls_pad);
    MPO_LAUNCH_CHECK();
    hipLaunchKernelGGL(zero_kernel, dim3((xrows + 255) / 256), dim3(256), 0, s, alpha, xrows);
    MPO_LAUNCH_CHECK();
    MPO_HIP(blocked_factor(xs, n, dp, amp, noise + kJitter, y_norm, Ab, Wb, Db, vb, L, W, alpha, info, s));
    const int T = np16 / 16;
    const size_t nw = wfrag_elems(np16);
    hipLaunchKernelGGL(zero_kernel, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, s, wfrag, (int)nw);
    MPO_LAUNCH_CHECK();
    hipLaunchKernelGGL(wave_plan_kernel, dim3(1), dim3(64), 0, s, T, wmeta);
    MPO_LAUNCH_CHECK();
    hipLaunchKernelGGL(pack_wfrag_kernel, dim3((4 * T * 64 + 255) / 256, T), dim3(256), 0, s, W, n, n, T, wmeta,
                       wfrag);
    MPO_LAUNCH_CHECK();
    // The expanded (MFMA) distance |c|^2 + |x|^2 - 2 c.x (d + 2 <= dp) carries an absolute
    // error of a few eps (|c|^2 + |x|^2) instead of the direct form's eps r2.  Its device
    // flag is set only when every |x|^2 <= kDistNorm and, scoring the observations
    // themselves both ways, (mu_n, q) agree within 1e-10; candidate tiles with some
    // |c|^2 > kDistNorm take the direct form in the kernel.  MPO_GP_DIST=0: never.
    const char* de = getenv("MPO_GP_DIST");
    const bool use_xb = d + 2 <= dp && !(de && de[0] == '0');
    bool xb_set = false;
    if (use_xb) {
        double* flag = xb + (size_t)xrows * dp;
        hipLaunchKernelGGL(xb_kernel, dim3(1), dim3(256), 0, s, xs, xrows, d, dp, xb);
        MPO_LAUNCH_CHECK();
        ScoreArgs sa{};
        sa.n = n; sa.np16 = np16; sa.T = T; sa.d = d;
        sa.amp = amp; sa.y_mean = y_mean; sa.y_std = y_std;
        sa.xs = xs; sa.ls = ls_pad; sa.alpha = alpha; sa.wfrag = wfrag; sa.wmeta = wmeta;
        sa.cand = X; sa.m = n; sa.flags = 1;
        const int nt = (n + kBM - 1) / kBM;
        const size_t lds = score_lds_bytes(dp, np16);
        sa.mq = mqc;                                   // direct form
        bool ok = launch_score_dp(dp, d, sa, nt, lds, s, false) == hipSuccess;
        sa.mq = mqc + 2 * (size_t)n;                   // expanded form
        sa.xb = xb;
        sa.xb_ok = flag;
        // a refused variant (MPO_GP_OCC forcing a spilling one) just leaves xb out
        ok = ok && launch_score_dp(dp, d, sa, nt, lds, s, false) == hipSuccess;
        if (ok) {
            hipLaunchKernelGGL(xb_check_kernel, dim3(1), dim3(256), 0, s, mqc, mqc + 2 * (size_t)n, alpha, n, amp,
                               flag);
            MPO_LAUNCH_CHECK();
        }
        xb_set = ok;
    }

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
    model->wmeta = wmeta;
    model->xb = xb_set ? xb : nullptr;
    return MPO_OK;
    MPO_GUARD_END
}

size_t mpo_gp_score_ws_bytes(const MpoGpModel* model, int64_t m, int k) {
    if (!model || m <= 0 || k < 0 || k > MPO_TOPK_MAX) return 0;
    if (!score_fits(model->dp, model->np16)) return 0;
    size_t used = 0;
    carve_score_ws(nullptr, m, k, &used);
    return used + 256;
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
    if (!score_fits(model->dp, model->np16)) { mpo::set_error("mpo_gp_acq_score: model too large"); return MPO_ENOTSUP; }
    const int64_t ntiles64 = (m + kBM - 1) / kBM;
    MPO_CHECK_ARG(ntiles64 < (1LL << 31), "mpo_gp_acq_score: too many candidates");
    const int ntiles = (int)ntiles64;
    const ScoreWs w = carve_score_ws(ws, m, k, nullptr);
    long long* part_idx = w.part_idx;
    double* part_val = w.part_val;
    long long* mid_idx = w.mid_idx;
    double* mid_val = w.mid_val;

    ScoreArgs a;
    a.n = model->n;
    a.np16 = model->np16;
    a.T = model->np16 / 16;
    a.d = model->d;
    a.amp = model->amp;
    a.y_mean = model->y_mean;
    a.y_std = model->y_std;
    a.xs = model->xs;
    a.xb = model->xb;
    a.xb_ok = model->xb ? model->xb + (size_t)(model->np16 + 32) * model->dp : nullptr;
    a.ls = model->ls;
    a.alpha = model->alpha;
    a.wfrag = model->wfrag;
    a.wmeta = model->wmeta;
    a.cand = cand;
    a.m = m;
    a.y_opt = y_opt;
    a.xi = xi;
    a.kappa = kappa;
    a.flags = flags;
    a.ei_positive = ei_positive;
    {
        const char* e = getenv("MPO_GP_DEBUG");
        a.dbg = e ? atoi(e) : 0;
    }
    a.mu = mu;
    a.sd = sd;
    a.vals = vals;
    a.k = k;
    a.part_idx = part_idx;
    a.part_val = part_val;
    a.mq = w.mq;   // FIN: the workgroup's own rows, finished inside the scoring kernel
    const size_t lds = score_lds_bytes(model->dp, model->np16);
    int grid = 0;
    MPO_HIP(launch_score_dp(model->dp, model->d, a, ntiles, lds, s, /*fin=*/true, &grid));
    const int nparts = 4 * grid;
    if (k > 0) {
        // stage 1: G groups of ~64 wave-lists each; stage 2: one list
        const int chunk = std::max(64, (nparts + kMergeGroups - 1) / kMergeGroups);
        const int G = (nparts + chunk - 1) / chunk;
        hipLaunchKernelGGL(topk_merge_kernel, dim3(G, 3), dim3(256), 0, s, part_idx, part_val, nparts, chunk, k,
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
    if (!score_fits(model->dp, model->np16)) { mpo::set_error("mpo_gp_ei_score: model too large"); return MPO_ENOTSUP; }
    const ScoreWs w = carve_score_ws(ws, m, 1, nullptr);
    long long* tidx = w.tail_idx;
    double* tval = w.tail_val;
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
    // dynamic LDS per point: 19 n doubles (16 waves) or 7 n (4 waves); the static
    // part (reduction rows, gradient tiles) is read from each kernel's code object
    static const size_t st16 = mpo::static_lds_bytes(reinterpret_cast<const void*>(acq_grad_kernel<16>));
    static const size_t st4 = mpo::static_lds_bytes(reinterpret_cast<const void*>(acq_grad_kernel<4>));
    const size_t lds16 = (size_t)19 * model->n * sizeof(double), lds4 = (size_t)7 * model->n * sizeof(double);
    const bool wide = lds16 + st16 <= kMaxLds;
    const size_t lds = wide ? lds16 : lds4;
    if (!wide && lds4 + st4 > kMaxLds) { mpo::set_error("mpo_gp_acq_grad: n=%d too large", model->n); return MPO_ENOTSUP; }
    auto kern = wide ? acq_grad_kernel<16> : acq_grad_kernel<4>;
    MPO_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(kern, dim3(batch), dim3(wide ? 1024 : 256), lds, static_cast<hipStream_t>(stream),
                       model->n, model->d, model->dp, model->amp, model->y_mean, model->y_std, model->xs, model->ls,
                       model->alpha, model->W, x, acq, y_opt, xi, kappa, f, g);
    MPO_LAUNCH_CHECK();
    return MPO_OK;
    MPO_GUARD_END
}

int mpo_gp_acq_grad_host(const MpoGpModel* model, const double* x_host, int batch, const int32_t* acq_host,
                         double y_opt, double xi, double kappa, double* f_host, double* g_host, void* stream) {
    MPO_GUARD_BEGIN
    MPO_CHECK_ARG(x_host && acq_host && f_host && g_host, "mpo_gp_acq_grad_host: null pointer");
    mpo::StreamDeviceScope on_device(static_cast<hipStream_t>(stream));
    auto dev_view = [](const void* h) -> void* {
        hipPointerAttribute_t at{};
        if (hipPointerGetAttributes(&at, h) != hipSuccess || at.type != hipMemoryTypeHost || !at.devicePointer) {
            (void)hipGetLastError();
            return nullptr;
        }
        return at.devicePointer;
    };
    void* xd = dev_view(x_host);
    void* ad = dev_view(acq_host);
    void* fd = dev_view(f_host);
    void* gd = dev_view(g_host);
    MPO_CHECK_ARG(xd && ad && fd && gd, "mpo_gp_acq_grad_host: buffers must be pinned host memory");
    const int rc = mpo_gp_acq_grad(model, static_cast<const double*>(xd), batch, static_cast<const int32_t*>(ad), y_opt,
                                   xi, kappa, static_cast<double*>(fd), static_cast<double*>(gd), stream);
    if (rc != MPO_OK) return rc;
    MPO_HIP(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
    return MPO_OK;
    MPO_GUARD_END
}

}  // extern "C"
