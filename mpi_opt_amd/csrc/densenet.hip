// densenet.hip -- the DenseNet population engine for gfx950.
//
// Replaces the per-trial Keras training of DenseNet (/root/reference/densenet.py:135-196,
// compiled by base_model.py:61-72 / mpiLAPI.py:197-201 and trained per MPI block by
// process_block.py:71-96) with one device-resident population: every member is a
// (trial, fold) with the SAME architecture (the reference grid fixes depth 10,
// 3 blocks, growth 12, nb_filter 16, dropout 0 and searches lr only,
// base_model.py:84-92), so every tensor of every member has one shape and the
// member index is just the outermost grid dimension of each launch.
//
// Layout (fp32, NHWC, member-major per buffer):
//   cat[s]  [B][H_s][W_s][C_s]  the dense-block concat of stage s: the initial conv /
//           pooled transition writes channels [0, f0), dense layer l writes its growth
//           slice [coff_l, coff_l + g) -- concatenation costs nothing;
//   dcat[s] gradient of cat[s]; the transition / head BN-backward STORES [0, C_s)
//           first, the dense layers then ACCUMULATE into [0, cin_l) last-to-first;
//   z[i]    [B][H][W][cin_i] = ELU(BN(cat[..., :cin_i])) of BN site i (the conv input,
//           kept for the weight gradient and the ELU derivative);
//   t[i]    transition conv output before AvgPool2.
//
// Kernels (all member-batched; MFMA = v_mfma_f32_16x16x4_f32, exact f32):
//   dn_conv<KS, NT>   implicit-GEMM 'same' conv, M = row-chunk pixels (<=128), N = cout,
//                     K = KS^2 * cin4: input rows + halo staged once in LDS, weights
//                     streamed from L2 one 16-k group ahead.  Also the input gradient
//                     (a 'same' conv of dOut with the rotated/transposed kernel).
//   dn_wgrad<KS, NT>  M = KS^2 * cin weight rows, N = cout, K = pixels of a sample
//                     group; partial slabs per group, reduced in fixed order.
//   dn_bn_stats / dn_bn_apply, dn_bn_bwd_reduce / dn_bn_bwd_apply
//                     BatchNormalization(axis=1) of NHWC = statistics per image ROW h:
//                     fp64 partial sums per (member, h, batch slice), folded in fixed
//                     order by the per-(sample, row) apply kernels (BN + ELU forward,
//                     BN/ELU backward into dcat).
//   dn_pool_fwd/bwd, dn_head_fwd/reduce (GAP + dense + softmax + categorical CE),
//   dn_adam (Keras Adam + l2 1e-4 gradient), dn_prep (padded weight copies).
#include "mpo_internal.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <vector>

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr float kBnEps = 1e-3f;
constexpr float kBnMomentum = 0.99f;
constexpr float kL2 = 1e-4f;
constexpr float kCeEps = 1e-7f;
constexpr int kWRowsSlack = 48;   // zero weight rows past K16 (the loop reads 2 groups ahead)
constexpr int kKoffSlack = 64;    // zero tap offsets past K16 (3 groups ahead)
constexpr int kMaxPix = 128;      // pixels per conv / wgrad workgroup chunk

__host__ __device__ constexpr inline int r4(int x) { return (x + 3) & ~3; }
__host__ __device__ constexpr inline int r16(int x) { return (x + 15) & ~15; }
// conv LDS pixel stride = cin4 + 2 == 2 (mod 4): lanes 0-15 (16 pixels, one channel)
// and lanes 16-31 (the next channel) land on the even / odd banks.
__host__ __device__ constexpr inline int conv_cp(int cin) { return r4(cin) + 2; }
// wgrad LDS pixel stride == 16 (mod 32): lanes 0-15 read 16 channels, lanes 16-31
// the next pixel -> banks 0-15 / 16-31.
__host__ __device__ constexpr inline int wg_cp(int c) { return c + ((48 - (c & 31)) & 31); }
// wgrad dOut pixel stride == 16 (mod 32)
__host__ __device__ constexpr inline int wg_ns(int nt) { return nt * 16 + ((nt & 1) ? 0 : 16); }

// ---- argument blocks ----------------------------------------------------------
struct ConvArgs {
    const float* in; long long in_ms; int in_ps;          // input (+ channel offset), member / pixel strides
    const float* bnc; long long bnc_ms;                   // BN site coef [4][H] (scale, shift at 2H, 3H): the
                                                          // input is cat and the conv sees ELU(x scale + shift)
    const int* order; long long ord_ms; long long row0;   // sample gather (initial conv only)
    long long img_floats;
    const float* w; long long w_ms;                       // padded weights [K16 + slack][N16]
    float* out; long long out_ms; int out_ps;
    int H, W, Cin, N, R;
    int pool;      // 1: out is AvgPool2D((2,2)) of the conv output, [B][H/2][W/2] (R, y0 even)
    int c1x1;      // 1x1 convs: dn_conv1x1_kernel where it applies (DnPlan::conv1x1)
    // r06: the BN backward reduce of the input gradient's consumer, in the epilogue (rpart
    // != nullptr): x = cat at the BN site (rx), its coef [4][H] (rcoef); per (sample,
    // 16-pixel row segment, row) the (sum dy, sum dy xhat) pair into rpart as dn_bn_bwd
    // slice partials (slice = b * SL + segment, SL = max(1, W / 16), rS slices)
    const float* rx; long long rx_ms; int rx_ps;
    const float* rcoef; long long rcoef_ms;
    double* rpart; int rS;
};

struct WgArgs {
    const float* in; long long in_ms; int in_ps;
    const float* bnc; long long bnc_ms;                   // as ConvArgs::bnc
    const int* order; long long ord_ms; long long row0;
    long long img_floats;
    const float* dout; long long dout_ms; int dout_ps;
    float* part; long long part_ms;                       // [G][Kw][N]
    int H, W, Cin, N, R, spg, B;
    int kw;        // dn_wgrad3: k-step interleave inside the workgroup (wg3_kw), 1 for dn_wgrad1
};

struct BnArgs {
    const float* x; long long x_ms; int x_ps;             // cat (channels [0, Cin))
    float* z; long long z_ms;                             // [B][H][W][Cin]
    float* coef; long long coef_ms;                       // [4][H]: mean, inv, scale = gamma inv, shift = beta - mean scale
    const float* params; long long p_ms; long long g_off, b_off;
    float* state; long long s_ms; long long mm_off, mv_off;
    float* grads;                                         // member stride p_ms
    const float* dz; long long dz_ms;                     // [B][H][W][Cin] (bcast == 0)
    const float* dg; long long dg_ms; float inv_hw;       // [B][Cin] / (H W)  (bcast == 1)
    float* dx; long long dx_ms; int dx_ps;
    int B, H, W, Cin, train, bcast, accumulate;
    int c0;        // dn_bn_stats reads channels [c0, Cin) (the growth slices new since the previous site)
    int prev;      // dn_bn_coef adds the previous site's totals (tot) to the slice partials
    double* tot;   // folded (sum, sum of squares) per (member, h): [n][H][2]
};

// ---- shared reductions -----------------------------------------------------------
// e = q*C + c walked by a fixed step (one division per thread, not per element)
struct Walk2 {
    int q, c, sq, sc, C;
    __device__ __forceinline__ Walk2(int e, int C_, int step) : C(C_) {
        q = e / C_;
        c = e - q * C_;
        sq = step / C_;
        sc = step - sq * C_;
    }
    __device__ __forceinline__ void next() {
        c += sc;
        q += sq;
        if (c >= C) { c -= C; ++q; }
    }
};

// e = (r*W + x)*C + c walked by a fixed step with mixed-radix adds: the staging loops
// divide once per thread instead of twice per element
struct Walk3 {
    int r, x, c, sr, sx, sc, W, C;
    __device__ __forceinline__ Walk3(int e, int W_, int C_, int step) : W(W_), C(C_) {
        const int p = e / C_, ps = step / C_;
        c = e - p * C_;
        r = p / W_;
        x = p - r * W_;
        sc = step - ps * C_;
        sr = ps / W_;
        sx = ps - sr * W_;
    }
    __device__ __forceinline__ void next() {
        c += sc;
        x += sx;
        r += sr;
        if (c >= C) { c -= C; ++x; }
        if (x >= W) { x -= W; ++r; }
    }
};

// z = ELU(BN(x)) of one element of image row h: the BN sites' conv / wgrad inputs
// and their backward's ELU' are formed from cat on the fly, so z is never stored
// (dn_bn_coef_kernel writes scale / shift).  ELU as TensorFlow's Elu kernel forms
// it, exp(y) - 1 (not expm1), on the hardware exp: every consumer re-forms z, so
// it must be cheap (expm1f here cost the conv and wgrad staging 10-35%).
__device__ __forceinline__ float bn_elu(float x, float s, float t) {
    const float y = x * s + t;
    // exp of min(y, 0) on every lane and a select (not a branch around the exp for
    // lanes with y <= 0): the same values, NaN included, and no exec-masked blocks
    const float e = __expf(y > 0.f ? 0.f : y) - 1.f;
    return y > 0.f ? y : e;
}

__device__ __forceinline__ double block_sum(double v, double* red) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) red[wave] = v;
    __syncthreads();
    double s = 0.0;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += red[i];
    return s;
}

// elements per thread in flight in the conv / wgrad LDS staging loops
constexpr int kStageU = 4;
constexpr int kWgStageU = 1;   // dn_wgrad3: more would cost it an occupancy step (> 128 VGPRs)

// ============================================================================
// Implicit-GEMM 'same' convolution, stride 1 (forward and input gradient).
// One workgroup = (member, sample b, output rows [y0, y0 + R)); M = R*W <= 128
// pixels in up to 8 m-tiles of 16 (2 per wave), N = NT tiles of 16.
// ============================================================================
template <int MT, int NT>
__device__ __forceinline__ void dn_conv_loop(const float* __restrict__ img, const int* __restrict__ koff,
                                             const float* __restrict__ Wt, int N16, int ngroups, const int (&pb)[2],
                                             f32x4 (&acc)[2][NT], int krow, int kcol) {
    const float* wsrc = Wt + krow * N16 + kcol;
    const int* kp = koff + krow * 4;
    float b0[4][NT], b1[4][NT], a0[4][MT], a1[4][MT];
    auto loadB = [&](int g, float (&dst)[4][NT]) {
        const float* src = wsrc + (long long)g * 16 * N16;
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int j = 0; j < NT; ++j) dst[u][j] = src[u * 4 * N16 + j * 16];
    };
    auto kof = [&](int g) { return *reinterpret_cast<const int4*>(kp + g * 16); };
    auto readA = [&](const int4 ko, float (&dst)[4][MT]) {
        const int kov[4] = {ko.x, ko.y, ko.z, ko.w};
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int i = 0; i < MT; ++i) dst[u][i] = img[pb[i] + kov[u]];
    };
    auto mma = [&](const float (&av)[4][MT], const float (&bw)[4][NT]) {
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int i = 0; i < MT; ++i)
#pragma unroll
                for (int j = 0; j < NT; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u][i], bw[u][j], acc[i][j], 0, 0, 0);
    };
    if constexpr (NT <= 2) {
        // narrow N (the growth convs): each group's MFMAs are few, so the weights
        // stream two groups ahead of their MFMAs (L2 latency) from a 3-buffer ring;
        // loads reach group ngroups + 1 (kWRowsSlack / kKoffSlack cover it)
        float b2[4][NT], a2[4][MT];
        loadB(0, b0);
        loadB(1, b1);
        int4 ko = kof(0);
        readA(ko, a0);
        ko = kof(1);
        for (int g = 0;; g += 3) {
            loadB(g + 2, b2);
            readA(ko, a1);
            ko = kof(g + 2);
            __builtin_amdgcn_sched_barrier(0);
            mma(a0, b0);
            __builtin_amdgcn_sched_barrier(0);
            if (g + 1 >= ngroups) break;
            loadB(g + 3, b0);
            readA(ko, a2);
            ko = kof(g + 3);
            __builtin_amdgcn_sched_barrier(0);
            mma(a1, b1);
            __builtin_amdgcn_sched_barrier(0);
            if (g + 2 >= ngroups) break;
            loadB(g + 4, b1);
            readA(ko, a0);
            ko = kof(g + 4);
            __builtin_amdgcn_sched_barrier(0);
            mma(a2, b2);
            __builtin_amdgcn_sched_barrier(0);
            if (g + 3 >= ngroups) break;
        }
        return;
    }
    loadB(0, b0);
    int4 ko = kof(0);
    readA(ko, a0);
    ko = kof(1);
    // two 16-k groups per iteration (an odd count runs one zero group from the slack)
    for (int g = 0; g < ngroups; g += 2) {
        loadB(g + 1, b1);
        readA(ko, a1);
        ko = kof(g + 2);
        __builtin_amdgcn_sched_barrier(0);
        mma(a0, b0);
        __builtin_amdgcn_sched_barrier(0);
        loadB(g + 2, b0);
        readA(ko, a0);
        ko = kof(g + 3);
        __builtin_amdgcn_sched_barrier(0);
        mma(a1, b1);
        __builtin_amdgcn_sched_barrier(0);
    }
}

template <int KS, int NT>
__global__ __launch_bounds__(256) void dn_conv_kernel(ConvArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    constexpr int P = (KS - 1) / 2;
    const int m = blockIdx.z, b = blockIdx.y, y0 = blockIdx.x * a.R;
    const int H = a.H, W = a.W, Cin = a.Cin;
    const int rows_out = min(a.R, H - y0);
    const int Wp = W + KS - 1;
    const int Cin4 = r4(Cin), Cp = conv_cp(Cin);
    const int rows = a.R + KS - 1;
    const float* src = a.order ? a.in + (long long)a.order[m * a.ord_ms + a.row0 + b] * a.img_floats
                               : a.in + m * a.in_ms + (long long)b * H * W * a.in_ps;
    float* img = smem;
    const int row_elems = Wp * Cp;
    const int img_elems = rows * row_elems;
    int* koff = reinterpret_cast<int*>(smem + r4(img_elems));
    const int K = KS * KS * Cin4, K16 = r16(K);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int krow = lane >> 4, kcol = lane & 15;

    const float* bnc = a.bnc ? a.bnc + m * a.bnc_ms : nullptr;
    // Staging: kStageU elements per thread in flight -- the loads are unconditional
    // (out-of-image taps read a clamped in-bounds address) and the zero padding is
    // selected when the value is used, so a thread issues kStageU loads before its
    // first wait instead of one load per dependent round trip.
    const bool vin = ((Cin & 3) == 0) && ((a.in_ps & 3) == 0) && ((reinterpret_cast<uintptr_t>(src) & 15) == 0);
    if (vin) {
        // float4 channel groups; the padding channels [Cin, Cp) are never read by
        // the k loop (koff covers c < Cin4 == Cin), so only the halo is zeroed
        const int C4 = Cin >> 2, tot = rows * Wp * C4;
        Walk3 wk(tid, Wp, C4, 256);
        for (int e0 = tid; e0 < tot; e0 += kStageU * 256) {
            float4 v[kStageU];
            float sc[kStageU], sh[kStageU];
            int dst[kStageU];
            bool ok[kStageU];
#pragma unroll
            for (int u = 0; u < kStageU; ++u) {
                const int gy = y0 + wk.r - P, gx = wk.x - P;
                ok[u] = e0 + u * 256 < tot && gy >= 0 && gy < H && gx >= 0 && gx < W;
                const int cy = ok[u] ? gy : 0, cx = ok[u] ? gx : 0, c4 = ok[u] ? wk.c : 0;
                v[u] = *reinterpret_cast<const float4*>(src + ((long long)cy * W + cx) * a.in_ps + 4 * c4);
                if (bnc) {
                    sc[u] = bnc[2 * H + cy];
                    sh[u] = bnc[3 * H + cy];
                }
                dst[u] = e0 + u * 256 < tot ? (wk.r * Wp + wk.x) * Cp + 4 * wk.c : -1;
                wk.next();
            }
#pragma unroll
            for (int u = 0; u < kStageU; ++u) {
                float4 x = v[u];
                if (bnc)
                    x = make_float4(bn_elu(x.x, sc[u], sh[u]), bn_elu(x.y, sc[u], sh[u]), bn_elu(x.z, sc[u], sh[u]),
                                    bn_elu(x.w, sc[u], sh[u]));
                if (!ok[u]) x = make_float4(0.f, 0.f, 0.f, 0.f);   // zero padding stays zero
                if (dst[u] >= 0) {   // Cp even: 8-byte aligned pairs
                    *reinterpret_cast<float2*>(img + dst[u]) = make_float2(x.x, x.y);
                    *reinterpret_cast<float2*>(img + dst[u] + 2) = make_float2(x.z, x.w);
                }
            }
        }
    } else {
        Walk3 wk(tid, Wp, Cp, 256);
        for (int e0 = tid; e0 < img_elems; e0 += kStageU * 256) {
            float v[kStageU], sc[kStageU], sh[kStageU];
            bool ok[kStageU];
#pragma unroll
            for (int u = 0; u < kStageU; ++u) {
                const int gy = y0 + wk.r - P, gx = wk.x - P;
                ok[u] = e0 + u * 256 < img_elems && gy >= 0 && gy < H && gx >= 0 && gx < W && wk.c < Cin;
                const int cy = ok[u] ? gy : 0, cx = ok[u] ? gx : 0, c = ok[u] ? wk.c : 0;
                v[u] = src[((long long)cy * W + cx) * a.in_ps + c];
                if (bnc) {
                    sc[u] = bnc[2 * H + cy];
                    sh[u] = bnc[3 * H + cy];
                }
                wk.next();
            }
#pragma unroll
            for (int u = 0; u < kStageU; ++u) {
                float x = v[u];
                if (bnc) x = bn_elu(x, sc[u], sh[u]);
                if (e0 + u * 256 < img_elems) img[e0 + u * 256] = ok[u] ? x : 0.f;
            }
        }
    }
    // tap offsets, each 16-k group stored as [krow][u] so a lane reads its four
    // k-steps (k = g*16 + u*4 + krow) as one b128
    for (int kq = tid; kq < K16 + kKoffSlack; kq += 256) {
        const int kk = (kq & ~15) + ((kq & 3) << 2) + ((kq >> 2) & 3);
        int off = 0;
        if (kk < K) {
            const int tap = kk / Cin4, c = kk - tap * Cin4;
            const int ky = tap / KS, kx = tap - ky * KS;
            off = (ky * Wp + kx) * Cp + c;
        }
        koff[kq] = off;
    }
    const int Mc = rows_out * W;
    const int mtiles = (Mc + 15) >> 4;
    const int mine = __builtin_amdgcn_readfirstlane(mtiles > wave + 4 ? 2 : (mtiles > wave ? 1 : 0));
    int pb[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int mm = (wave + 4 * i) * 16 + (lane & 15);
        pb[i] = mm < Mc ? ((mm / W) * Wp + (mm % W)) * Cp : 0;
    }
    f32x4 acc[2][NT];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    __syncthreads();
    const int ngroups = K16 >> 4;
    const float* Wt = a.w + m * a.w_ms;
    const int N16 = NT * 16;
    if (mine == 2) dn_conv_loop<2, NT>(img, koff, Wt, N16, ngroups, pb, acc, krow, kcol);
    else if (mine == 1) dn_conv_loop<1, NT>(img, koff, Wt, N16, ngroups, pb, acc, krow, kcol);
    else if (!a.pool) return;

    if (a.pool) {
        // the transition's AvgPool2 in the epilogue (the pre-pool output never goes to
        // HBM): the chunk's outputs through the LDS, then each pooled element as
        // dn_pool_fwd forms it, 0.25 (x00 + x01 + x10 + x11)
        constexpr int S = NT * 16 + 4;
        float* ot = smem;
        __syncthreads();   // every wave is done with img / koff
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            if (i >= mine) break;
            const int mt = wave + 4 * i;
#pragma unroll
            for (int j = 0; j < NT; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) ot[(mt * 16 + krow * 4 + r) * S + j * 16 + kcol] = acc[i][j][r];
        }
        __syncthreads();
        const int H2 = H / 2, W2 = W / 2, pr0 = y0 / 2;
        const int npr = min(rows_out / 2, H2 - pr0);
        float* dst = a.out + m * a.out_ms + ((long long)b * H2 + pr0) * W2 * a.out_ps;
        for (int e = tid; e < npr * W2 * a.N; e += 256) {
            const int q = e / a.N, n = e - q * a.N;
            const int pr = q / W2, px = q - pr * W2;
            const float* s0 = ot + (2 * pr * W + 2 * px) * S + n;
            dst[((long long)pr * W2 + px) * a.out_ps + n] = 0.25f * (s0[0] + s0[S] + s0[W * S] + s0[W * S + S]);
        }
        return;
    }

    float* dst = a.out + m * a.out_ms + ((long long)b * H + y0) * W * a.out_ps;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        if (i >= mine) break;
        const int mt = wave + 4 * i;
#pragma unroll
        for (int j = 0; j < NT; ++j) {
            const int n = j * 16 + kcol;
            if (n >= a.N) continue;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int mm = mt * 16 + krow * 4 + r;
                if (mm < Mc) dst[(long long)mm * a.out_ps + n] = acc[i][j][r];
            }
        }
    }
    if (a.rpart) {
        // the consumer's dn_bn_bwd_reduce on the values just produced (dz = this output):
        // dy = dz ELU'(x scale + shift), sums of dy and dy xhat per image row -- a lane's
        // four pixels share a row (W % 4 == 0); a 16-pixel tile is one row segment for
        // W >= 16, 16 / W whole rows below; one (b, segment, row) slot per tile and row
        const float* xr = a.rx + m * a.rx_ms + ((long long)b * H + y0) * W * a.rx_ps;
        const float* cf = a.rcoef + m * a.rcoef_ms;
        const int SL = W >= 16 ? W / 16 : 1;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            if (i >= mine) break;
            const int mt = wave + 4 * i;
            const int mm0 = mt * 16 + krow * 4;
            double sdy = 0.0, sdyx = 0.0;
            if (mm0 < Mc) {
                const int h = y0 + mm0 / W;
                const float mean = cf[h], inv = cf[H + h], bs_ = cf[2 * H + h], bt_ = cf[3 * H + h];
#pragma unroll
                for (int j = 0; j < NT; ++j) {
                    const int n = j * 16 + kcol;
                    if (n >= a.N) continue;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float xv = xr[(long long)(mm0 + r) * a.rx_ps + n];
                        const float y = xv * bs_ + bt_;
                        const float dy = acc[i][j][r] * (y > 0.f ? 1.f : __expf(y));
                        const float xh = (xv - mean) * inv;
                        sdy += dy;
                        sdyx += (double)dy * xh;
                    }
                }
            }
            const int tr = W >= 16 ? 1 : 16 / W;
            for (int q = 0; q < tr; ++q) {
                const bool row_q = W >= 16 || (krow * 4) / W == q;
                double v0 = row_q ? sdy : 0.0, v1 = row_q ? sdyx : 0.0;
#pragma unroll
                for (int off = 32; off >= 1; off >>= 1) {
                    v0 += __shfl_xor(v0, off);
                    v1 += __shfl_xor(v1, off);
                }
                const int pix = mt * 16 + q * W;   // the row's first pixel in this tile
                if (lane == 0 && pix < Mc) {
                    const int slot = W >= 16 ? (pix % W) / 16 : 0;
                    double* o = a.rpart + (((long long)m * a.rS + ((long long)b * SL + slot)) * H + (y0 + pix / W)) * 2;
                    o[0] = v0;
                    o[1] = v1;
                }
            }
        }
    }
}

// ============================================================================
// 1x1 convolution (the transitions: forward with BN + ELU and the AvgPool2 epilogue,
// and the input gradient), streamed without LDS staging (r05).  K = cin is small
// (40, 64 at the reference config), so dn_conv_kernel's per-workgroup staging and
// barriers dominated it (conv<1, 3>: 0.36 ms per launch, 2.7x the HBM time).  Here
// a wave owns a 2 x 8 pixel patch: lane (t = l % 16, q = l / 16) loads pixel t's
// channels [16 v + 4 q, +4) as one float4 per 16-channel block v, applies BN + ELU
// in registers, and component i of block v is MFMA k-step (v, i) over the channels
// {16 v + 4 q' + i}; the B rows are the same channels.  Every load of the wave is
// issued before its first MFMA.  The pooled epilogue adds the 2 x 2 neighbours
// across lanes l and l + 32 in dn_pool_fwd's order, ((x00 + x01) + x10) + x11.
// ============================================================================
template <int NT, int CB, bool POOL>
__global__ __launch_bounds__(256) void dn_conv1x1_kernel(ConvArgs a) {
    const int m = blockIdx.z, b = blockIdx.y;
    const int H = a.H, W = a.W, Cin = a.Cin;
    const int lane = threadIdx.x & 63;
    const int tile = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int tw = W >> 3, ntile = (H >> 1) * tw;
    if (tile >= ntile) return;
    const int h0 = 2 * (tile / tw), w0 = 8 * (tile % tw);
    const int t = lane & 15, q = lane >> 4;
    const int hy = h0 + (t >> 3), wx = w0 + (t & 7);
    const float* src = a.in + m * a.in_ms + (((long long)b * H + hy) * W + wx) * a.in_ps;
    float4 xv[CB];
#pragma unroll
    for (int v = 0; v < CB; ++v) {
        const int c = 16 * v + 4 * q;
        xv[v] = *reinterpret_cast<const float4*>(src + min(c, (Cin - 4) & ~3));   // clamped, zeroed below
    }
    const float* Wt = a.w + m * a.w_ms;
    constexpr int N16 = NT * 16;
    float bw[CB][4][NT];
#pragma unroll
    for (int v = 0; v < CB; ++v)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < NT; ++j) bw[v][i][j] = Wt[(16 * v + 4 * q + i) * N16 + 16 * j + t];
    float sc = 1.f, sh = 0.f;
    if (a.bnc) {
        const float* bnc = a.bnc + m * a.bnc_ms;
        sc = bnc[2 * H + hy];
        sh = bnc[3 * H + hy];
    }
    f32x4 acc[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int v = 0; v < CB; ++v) {
        const int c = 16 * v + 4 * q;
        float z[4] = {xv[v].x, xv[v].y, xv[v].z, xv[v].w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if (a.bnc) z[i] = bn_elu(z[i], sc, sh);
            if (c + i >= Cin) z[i] = 0.f;
#pragma unroll
            for (int j = 0; j < NT; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(z[i], bw[v][i][j], acc[j], 0, 0, 0);
        }
    }
    // C: lane (col n = 16 j + t, row group q) holds rows 4 q + r = patch pixels
    // (row (4 q + r) / 8, column (4 q + r) % 8)
    if constexpr (POOL) {
        const int H2 = H >> 1, W2 = W >> 1;
        float* dst = a.out + m * a.out_ms + ((long long)b * H2 + (h0 >> 1)) * W2 * a.out_ps;
#pragma unroll
        for (int j = 0; j < NT; ++j) {
            const int n = 16 * j + t;
            // lanes q = 0, 1 own the top row's pairs (r0, r1), (r2, r3); q + 2 the bottom row's
            const float lo0 = acc[j][0] + acc[j][1], lo1 = acc[j][2] + acc[j][3];
            const float b00 = __shfl_xor(acc[j][0], 32), b01 = __shfl_xor(acc[j][1], 32);
            const float b10 = __shfl_xor(acc[j][2], 32), b11 = __shfl_xor(acc[j][3], 32);
            if (q < 2 && n < a.N) {
                const int pc = (w0 >> 1) + 2 * q;   // pooled column of (r0, r1)
                dst[(long long)pc * a.out_ps + n] = 0.25f * ((lo0 + b00) + b01);
                dst[(long long)(pc + 1) * a.out_ps + n] = 0.25f * ((lo1 + b10) + b11);
            }
        }
    } else {
        float* dst = a.out + m * a.out_ms + ((long long)b * H * W) * a.out_ps;
#pragma unroll
        for (int j = 0; j < NT; ++j) {
            const int n = 16 * j + t;
            if (n >= a.N) continue;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int pt = 4 * q + r;
                const int py = h0 + (pt >> 3), px = w0 + (pt & 7);
                dst[((long long)py * W + px) * a.out_ps + n] = acc[j][r];
            }
        }
    }
}

// ============================================================================
// Weight gradient of a 3x3 'same' conv:
//   dW[(ky,kx,c)][n] = sum_{b,y,x} in[b][y+ky-1][x+kx-1][c] * dout[b][y][x][n]
// GEMM view M = 9 cin weight rows, N = cout, K = pixels.  One workgroup =
// (member, 768-row m-group, group of spg samples): 8 waves x up to 6 m-tiles, so
// every DenseNet layer of the reference grid (M <= 684) stages each input row
// chunk exactly once.  Per row chunk (<= 128 pixels) the input rows + halo and
// the dOut rows are staged in LDS; the zero halo columns / padding channels are
// written once per workgroup, the data with float4 loads when the channel
// counts allow (runtime-uniform branch).  One partial slab per sample group.
// Layers with few m-tiles (M = 9 cin <= 6 mw tiles) split the row chunk's k-steps
// over kw = 8 / mw wave groups instead (wave = kq * mw + wm: m-tiles wm, wm + mw,
// ..., k-steps kq, kq + kw, ...), so each wave keeps up to 6 independent MFMA chains
// over the LDS latency of its operand reads; at the end the k groups' accumulators
// are summed through the LDS in fixed order (kq = 0, 1, ...) into the one slab.
// ============================================================================
constexpr int kWgWaves = 8;
constexpr int kWgMT = 6;
constexpr int kWgRows = kWgWaves * kWgMT * 16;   // 768
// m-tiles per wave of the first m-group when mw waves share its tiles
__host__ __device__ inline int wg3_tpw(int Kw, int mw) {
    const int mt = min(kWgRows / 16, (Kw + 15) >> 4);
    return (mt + mw - 1) / mw;
}

template <int MT, int NT>
__device__ __forceinline__ void dn_wgrad_chunk(const float* __restrict__ img, const float* __restrict__ dl,
                                               const int* __restrict__ ptab, const int (&aoff)[kWgMT], int ns, int nk4,
                                               int s0, int ds, int krow, int kcol, f32x4 (&acc)[kWgMT][NT]) {
    float a0[MT], a1[MT], b0[NT], b1[NT];
    auto rd = [&](int s, float (&av)[MT], float (&bv)[NT]) {
        const int p = 4 * s + krow;
        const int po = ptab[p];
#pragma unroll
        for (int i = 0; i < MT; ++i) av[i] = img[aoff[i] + po];
#pragma unroll
        for (int j = 0; j < NT; ++j) bv[j] = dl[p * ns + j * 16 + kcol];
    };
    auto mma = [&](const float (&av)[MT], const float (&bv)[NT]) {
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int j = 0; j < NT; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i], bv[j], acc[i][j], 0, 0, 0);
    };
    // k-steps s0, s0 + ds, ... < nk4; s + ds < nk4 + kWgWaves: the tables hold
    // kWgWaves zero k-steps of slack
    rd(s0, a0, b0);
    for (int s = s0; s < nk4; s += 2 * ds) {
        rd(s + ds, a1, b1);
        __builtin_amdgcn_sched_barrier(0);
        mma(a0, b0);
        __builtin_amdgcn_sched_barrier(0);
        if (s + ds >= nk4) break;
        rd(s + 2 * ds, a0, b0);
        __builtin_amdgcn_sched_barrier(0);
        mma(a1, b1);
        __builtin_amdgcn_sched_barrier(0);
    }
}

template <int NT>
__global__ __launch_bounds__(kWgWaves * 64) void dn_wgrad3_kernel(WgArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    constexpr int KS = 3, P = 1;
    constexpr int NTH = kWgWaves * 64;
    const int m = blockIdx.z, grp = blockIdx.y, mg = blockIdx.x;
    const int H = a.H, W = a.W, Cin = a.Cin, N = a.N;
    const int Kw = KS * KS * Cin;
    const int Wp = W + KS - 1;
    const int Cp = wg_cp(Cin);
    const int ns = wg_ns(NT);
    const int R = a.R;
    const int rows = R + KS - 1;
    const int img_elems = rows * Wp * Cp;
    const int np = 4 * (((R * W + 3) >> 2) + kWgWaves);   // pixel slots incl. kWgWaves zero k-steps of slack
    float* img = smem;
    float* dl = smem + r4(img_elems);
    int* ptab = reinterpret_cast<int*>(dl + np * ns);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int krow = lane >> 4, kcol = lane & 15;
    const int mtiles = (Kw + 15) >> 4;
    const int t0 = mg * (kWgRows / 16);   // kw > 1 only when every tile fits one m-group
    const int kw = a.kw, mw = kWgWaves / kw;
    const int wm = wave % mw, kq = wave / mw;
    const int mine = __builtin_amdgcn_readfirstlane(min(kWgMT, max(0, (mtiles - t0 - wm + mw - 1) / mw)));

    int aoff[kWgMT];
#pragma unroll
    for (int i = 0; i < kWgMT; ++i) {
        const int r = (t0 + wm + mw * i) * 16 + (lane & 15);
        int off = 0;   // rows past Kw read finite LDS; their partials are never stored
        if (r < Kw) {
            const int tap = r / Cin, c = r - tap * Cin;
            const int ky = tap / KS, kx = tap - ky * KS;
            off = (ky * Wp + kx) * Cp + c;
        }
        aoff[i] = off;
    }
    // zero everything once: halo columns, padding channels and dOut padding stay zero
    for (int e = tid; e < r4(img_elems) + np * ns; e += NTH) smem[e] = 0.f;
    for (int p = tid; p < np; p += NTH) ptab[p] = p < R * W ? ((p / W) * Wp + (p % W)) * Cp : 0;
    f32x4 acc[kWgMT][NT];
#pragma unroll
    for (int i = 0; i < kWgMT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // vector staging when every row segment is float4-aligned (uniform)
    const bool vin = ((Cin & 3) == 0) && ((a.in_ps & 3) == 0) && !a.order &&
                     ((reinterpret_cast<uintptr_t>(a.in) & 15) == 0);
    const bool vdo = ((N & 3) == 0) && ((a.dout_ps & 3) == 0) && ((reinterpret_cast<uintptr_t>(a.dout) & 15) == 0);
    const int C4 = Cin >> 2, N4 = N >> 2;
    const int b0 = grp * a.spg, b1 = min(a.B, b0 + a.spg);
    const float* inm = a.in + m * a.in_ms;
    const float* dom = a.dout + m * a.dout_ms;
    const float* bnc = a.bnc ? a.bnc + m * a.bnc_ms : nullptr;
    for (int b = b0; b < b1; ++b) {
        const float* src = a.order ? a.in + (long long)a.order[m * a.ord_ms + a.row0 + b] * a.img_floats
                                   : inm + (long long)b * H * W * a.in_ps;
        for (int y0 = 0; y0 < H; y0 += R) {
            const int Mc = min(R, H - y0) * W;
            __syncthreads();   // the previous chunk's MFMAs are done with the LDS (and the zero fill)
            if (vin) {
                // kWgStageU float4 loads in flight per thread (clamped, zeroed when used)
                const int tot = rows * W * C4;
                Walk3 wk(tid, W, C4, NTH);
                for (int e0 = tid; e0 < tot; e0 += kWgStageU * NTH) {
                    float4 v[kWgStageU];
                    float sc[kWgStageU], sh[kWgStageU];
                    int dst[kWgStageU];
                    bool ok[kWgStageU];
#pragma unroll
                    for (int u = 0; u < kWgStageU; ++u) {
                        const int gy = y0 + wk.r - P;
                        ok[u] = e0 + u * NTH < tot && gy >= 0 && gy < H;
                        const int cy = ok[u] ? gy : 0, x = ok[u] ? wk.x : 0, c4 = ok[u] ? wk.c : 0;
                        v[u] = *reinterpret_cast<const float4*>(src + ((long long)cy * W + x) * a.in_ps + 4 * c4);
                        if (bnc) {
                            sc[u] = bnc[2 * H + cy];
                            sh[u] = bnc[3 * H + cy];
                        }
                        dst[u] = e0 + u * NTH < tot ? (wk.r * Wp + wk.x + P) * Cp + 4 * wk.c : -1;
                        wk.next();
                    }
#pragma unroll
                    for (int u = 0; u < kWgStageU; ++u) {
                        float4 x = v[u];
                        if (bnc)
                            x = make_float4(bn_elu(x.x, sc[u], sh[u]), bn_elu(x.y, sc[u], sh[u]),
                                            bn_elu(x.z, sc[u], sh[u]), bn_elu(x.w, sc[u], sh[u]));
                        if (!ok[u]) x = make_float4(0.f, 0.f, 0.f, 0.f);
                        if (dst[u] >= 0) *reinterpret_cast<float4*>(img + dst[u]) = x;
                    }
                }
            } else {
                const int tot = rows * W * Cin;
                Walk3 wk(tid, W, Cin, NTH);
                for (int e = tid; e < tot; e += NTH, wk.next()) {
                    const int r = wk.r, x = wk.x, c = wk.c;
                    const int gy = y0 + r - P;
                    float v = 0.f;
                    if (gy >= 0 && gy < H) {
                        v = src[((long long)gy * W + x) * a.in_ps + c];
                        if (bnc) v = bn_elu(v, bnc[2 * H + gy], bnc[3 * H + gy]);
                    }
                    img[(r * Wp + x + P) * Cp + c] = v;
                }
            }
            const float* dsrc = dom + ((long long)b * H + y0) * W * a.dout_ps;
            const int npix = R * W;   // rows past Mc are zeroed (the last chunk of a sample)
            if (vdo) {
                for (int e = tid; e < npix * N4; e += NTH) {
                    const int p = e / N4, n4 = e - p * N4;
                    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
                    if (p < Mc) v = *reinterpret_cast<const float4*>(dsrc + (long long)p * a.dout_ps + 4 * n4);
                    *reinterpret_cast<float4*>(dl + p * ns + 4 * n4) = v;
                }
            } else {
                for (int e = tid; e < npix * N; e += NTH) {
                    const int p = e / N, n = e - p * N;
                    dl[p * ns + n] = p < Mc ? dsrc[(long long)p * a.dout_ps + n] : 0.f;
                }
            }
            __syncthreads();
            const int nk4 = (Mc + 3) >> 2;
            switch (mine) {
                case 6: dn_wgrad_chunk<6, NT>(img, dl, ptab, aoff, ns, nk4, kq, kw, krow, kcol, acc); break;
                case 5: dn_wgrad_chunk<5, NT>(img, dl, ptab, aoff, ns, nk4, kq, kw, krow, kcol, acc); break;
                case 4: dn_wgrad_chunk<4, NT>(img, dl, ptab, aoff, ns, nk4, kq, kw, krow, kcol, acc); break;
                case 3: dn_wgrad_chunk<3, NT>(img, dl, ptab, aoff, ns, nk4, kq, kw, krow, kcol, acc); break;
                case 2: dn_wgrad_chunk<2, NT>(img, dl, ptab, aoff, ns, nk4, kq, kw, krow, kcol, acc); break;
                case 1: dn_wgrad_chunk<1, NT>(img, dl, ptab, aoff, ns, nk4, kq, kw, krow, kcol, acc); break;
                default: break;
            }
        }
    }
    if (kw > 1) {
        // one wave's accumulators: its m-tiles (kw > 1: one m-group, so wg3_tpw) x NT
        const int TS = wg3_tpw(Kw, mw) * NT * 256;
        __syncthreads();                       // the last chunk's MFMAs are done with the LDS
        if (kq > 0) {
            float* dst = smem + ((kq - 1) * mw + wm) * TS;
#pragma unroll
            for (int i = 0; i < kWgMT; ++i) {
                if (i >= mine) break;
#pragma unroll
                for (int j = 0; j < NT; ++j) *reinterpret_cast<f32x4*>(dst + (i * NT + j) * 256 + lane * 4) = acc[i][j];
            }
        }
        __syncthreads();
        if (kq > 0) return;
        for (int g = 1; g < kw; ++g) {
            const float* src = smem + ((g - 1) * mw + wm) * TS;
#pragma unroll
            for (int i = 0; i < kWgMT; ++i) {
                if (i >= mine) break;
#pragma unroll
                for (int j = 0; j < NT; ++j) {
                    const f32x4 v = *reinterpret_cast<const f32x4*>(src + (i * NT + j) * 256 + lane * 4);
#pragma unroll
                    for (int r = 0; r < 4; ++r) acc[i][j][r] += v[r];
                }
            }
        }
    }
    float* part = a.part + m * a.part_ms + (long long)grp * Kw * N;
#pragma unroll
    for (int i = 0; i < kWgMT; ++i) {
        if (i >= mine) break;
        const int mt = t0 + wm + mw * i;
#pragma unroll
        for (int j = 0; j < NT; ++j) {
            const int n = j * 16 + kcol;
            if (n >= N) continue;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = mt * 16 + krow * 4 + r;
                if (row < Kw) part[(long long)row * N + n] = acc[i][j][r];
            }
        }
    }
}

// ============================================================================
// Weight gradient of a 1x1 conv (the transitions): dW[c][n] = sum_p z[p][c] dout[p][n],
// a plain GEMM with tiny M = cin and N = cout and K = the group's pixels, which are
// contiguous in both operands.  Split-K inside the workgroup: every wave holds all
// MT x NT tiles and streams every 8th k-step straight from global memory (no LDS
// staging); the 8 partial accumulators are summed through LDS in fixed order.
// r04: the raw operands of kWg1Depth k-steps are in flight per wave (r03 had one:
// each k-step waited a full memory latency, 1.8 ms per 32-member launch at 5% of
// the MFMA rate), the image row of a pixel is tracked by adds instead of a
// division per k-step, and the BN (scale, shift) per row sits in the LDS; BN + ELU
// are applied when a k-step is consumed.  Same MFMA sequence per accumulator.
// ============================================================================
constexpr int kWg1Depth = 4;
constexpr int kWg1MaxH = 1024;   // image rows whose BN coefficients dn_wgrad1 keeps in LDS

template <int MT, int NT>
__global__ __launch_bounds__(kWgWaves * 64) void dn_wgrad1_kernel(WgArgs a) {
    __shared__ __attribute__((aligned(16))) float red[kWgWaves - 1][MT * NT * 4 * 64];
    __shared__ float bnl[2 * kWg1MaxH];
    const int m = blockIdx.z, grp = blockIdx.y;
    const int Cin = a.Cin, N = a.N;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int krow = lane >> 4, kcol = lane & 15;
    const int H = a.H, W = a.W, HW = H * W;
    const int b0 = grp * a.spg, b1 = min(a.B, b0 + a.spg);
    const long long p0 = (long long)b0 * HW, p1 = (long long)b1 * HW;
    const float* z = a.in + m * a.in_ms;
    const float* d = a.dout + m * a.dout_ms;
    const float* bnc = a.bnc ? a.bnc + m * a.bnc_ms : nullptr;
    if (bnc)
        for (int e = tid; e < 2 * H; e += kWgWaves * 64) bnl[e] = bnc[2 * H + e];   // scale rows, then shift rows
    __syncthreads();
    bool am[MT], bm[NT];
#pragma unroll
    for (int i = 0; i < MT; ++i) am[i] = i * 16 + kcol < Cin;
#pragma unroll
    for (int j = 0; j < NT; ++j) bm[j] = j * 16 + kcol < N;
    f32x4 acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // k-step s covers pixels [p0 + 4s, p0 + 4s + 4); wave w takes s = w, w + 8, ...:
    // this lane's pixel advances by 32 per k-step of the wave; its image row
    // h = (pixel / W) mod H is carried as (h, column) and advanced by adds
    const long long nsteps = (p1 - p0 + 3) >> 2;
    const long long pl0 = 4LL * wave + krow;                 // lane's pixel offset in the group
    int col = (int)(pl0 % W), hrow = (int)((pl0 / W) % H);   // once per kernel (b0 * HW is a multiple of W and H * W)
    const int dstep = 4 * kWgWaves;                          // pixels per wave k-step
    const int dcol = dstep % W, drow = dstep / W;
    float zr[kWg1Depth][MT], dr[kWg1Depth][NT];
    int hr[kWg1Depth];
    bool okr[kWg1Depth];
    // loads are unconditional (clamped to the last pixel / channel, the value zeroed
    // afterwards by a select), so every path has the same loads in flight and the
    // compiler's vmcnt waits stay kWg1Depth - 1 k-steps behind
    auto ld = [&](long long s, int slot) {
        const long long p = p0 + 4 * s + krow;
        const bool ok = p < p1;
        const long long pc = ok ? p : p1 - 1;
        okr[slot] = ok;
        hr[slot] = hrow;
        const float* zp = z + pc * a.in_ps;
        const float* dp = d + pc * a.dout_ps;
#pragma unroll
        for (int i = 0; i < MT; ++i) zr[slot][i] = zp[min(i * 16 + kcol, Cin - 1)];
#pragma unroll
        for (int j = 0; j < NT; ++j) dr[slot][j] = dp[min(j * 16 + kcol, N - 1)];   // raw: zeroed when used
        // the next k-step of this wave: pixel + 32 (selects, not branches)
        col += dcol;
        const bool wrap = col >= W;
        col = wrap ? col - W : col;
        hrow += drow + (wrap ? 1 : 0);
        hrow = hrow >= H ? hrow - H : hrow;
        if (drow + 1 >= H) hrow %= H;        // images of fewer than 32 pixels (uniform, rare)
    };
    auto use = [&](int slot) {
        float av[MT];
        // (scale, shift) = (1, 0) and no ELU without BN; a padding lane's value is zero
        const float sc = bnc ? bnl[hr[slot]] : 1.f, sh = bnc ? bnl[H + hr[slot]] : 0.f;
#pragma unroll
        for (int i = 0; i < MT; ++i) {
            const float v = bn_elu(zr[slot][i], sc, sh);
            av[i] = (okr[slot] && am[i]) ? (bnc ? v : zr[slot][i]) : 0.f;
        }
        float bv[NT];
#pragma unroll
        for (int j = 0; j < NT; ++j) bv[j] = (okr[slot] && bm[j]) ? dr[slot][j] : 0.f;
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int j = 0; j < NT; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i], bv[j], acc[i][j], 0, 0, 0);
    };
    // this wave's k-steps t = 0 .. nw-1 (s = wave + 8 t), kWg1Depth in flight; the loop
    // runs whole groups of kWg1Depth: steps past nw are all padding lanes (zero A and
    // B), exact no-ops on the accumulators
    const long long nw = nsteps > wave ? (nsteps - wave + kWgWaves - 1) / kWgWaves : 0;
#pragma unroll
    for (int u = 0; u < kWg1Depth; ++u) ld(wave + (long long)kWgWaves * u, u);
    for (long long t = 0; t < nw; t += kWg1Depth) {
#pragma unroll
        for (int u = 0; u < kWg1Depth; ++u) {
            use(u);
            ld(wave + (long long)kWgWaves * (t + u + kWg1Depth), u);
        }
    }
    if (wave > 0) {
        float* r = red[wave - 1];
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int j = 0; j < NT; ++j)
#pragma unroll
                for (int q = 0; q < 4; ++q) r[((i * NT + j) * 4 + q) * 64 + lane] = acc[i][j][q];
    }
    __syncthreads();
    if (wave != 0) return;
    float* part = a.part + m * a.part_ms + (long long)grp * Cin * N;
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                float v = acc[i][j][q];
                for (int w = 0; w < kWgWaves - 1; ++w) v += red[w][((i * NT + j) * 4 + q) * 64 + lane];
                const int row = i * 16 + krow * 4 + q, n = j * 16 + kcol;
                if (row < Cin && n < N) part[(long long)row * N + n] = v;
            }
}

// grads[w_off + e] = sum_g part[g][e]  (fixed order: deterministic)
__global__ void dn_wgrad_reduce_kernel(const float* __restrict__ part, long long part_ms, int G, long long cnt,
                                       float* __restrict__ grads, long long g_ms, long long w_off) {
    const int m = blockIdx.y;
    const float* pm = part + m * part_ms;
    for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < cnt; e += (long long)gridDim.x * blockDim.x) {
        float s = 0.f;
        for (int g = 0; g < G; ++g) s += pm[g * cnt + e];
        grads[m * g_ms + w_off + e] = s;
    }
}

// Padded weight copies.  Forward: dst[(tap*cin4 + c)][n] = w[tap][c][n].
// Input gradient (transpose = 1): dst[(tap'*cout4 + f)][c] = w[KS^2-1-tap'][c][f].
__global__ void dn_prep_kernel(const float* __restrict__ params, long long p_ms, long long w_off, float* __restrict__ dst,
                               long long d_ms, int taps, int cin, int cout, int rows, int n16, int transpose) {
    const int m = blockIdx.y;
    const float* w = params + m * p_ms + w_off;
    float* d = dst + m * d_ms;
    const int total = rows * n16;
    for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
        const int k = e / n16, n = e - k * n16;
        float v = 0.f;
        if (!transpose) {
            const int c4 = r4(cin), tap = k / c4, c = k - tap * c4;
            if (tap < taps && c < cin && n < cout) v = w[((long long)tap * cin + c) * cout + n];
        } else {
            const int f4 = r4(cout), tp = k / f4, f = k - tp * f4;
            if (tp < taps && f < cout && n < cin) v = w[((long long)(taps - 1 - tp) * cin + n) * cout + f];
        }
        d[e] = v;
    }
}

// ============================================================================
// BatchNormalization(mode=0, axis=1) of an NHWC tensor: statistics per image row h
// over (batch, W, channels) -- densenet.py:24-27 -- then ELU.
//   dn_bn_stats  grid (h, batch slice, member): fp64 (sum, sum of squares) of the
//                slice's (b, w, c) elements of row h -> part[member][slice][h][2];
//   dn_bn_apply  grid (b*H + h, member): folds the S slice partials in fixed order
//                (deterministic), z = ELU(x * gamma inv + (beta - mean gamma inv)).
//                Training: block (b = 0) stores mean / inv and updates the moving
//                averages; evaluation: the moving averages.
// ============================================================================
// V = 4: rows walked as float4 (Cin, the pixel strides and every base 16-B
// aligned -- bn_vec4 on the host); V = 1 otherwise.
template <int V>
__device__ __forceinline__ void ldv(const float* p, float (&v)[V]) {
    if constexpr (V == 4) {
        const float4 t = *reinterpret_cast<const float4*>(p);
        v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
    } else {
        v[0] = *p;
    }
}

template <int V>
__device__ __forceinline__ void stv(float* p, const float (&v)[V]) {
    if constexpr (V == 4) *reinterpret_cast<float4*>(p) = float4{v[0], v[1], v[2], v[3]};
    else *p = v[0];
}

template <int V>
__global__ __launch_bounds__(256) void dn_bn_stats_kernel(BnArgs a, double* __restrict__ part, int S, int bs) {
    __shared__ double red[4];
    const int h = blockIdx.x, sl = blockIdx.y, m = blockIdx.z, tid = threadIdx.x;
    const int H = a.H, W = a.W, Cv = (a.Cin - a.c0) / V;
    const int rowv = W * Cv;
    const long long bstride = (long long)H * W * a.x_ps;
    const float* xm = a.x + m * a.x_ms + (long long)h * W * a.x_ps + a.c0;
    const int b0 = sl * bs, b1 = min(a.B, b0 + bs);
    double s = 0.0, q = 0.0;
    // (sample, pixel, channel group) flattened: every thread busy even for a
    // 12-channel slice, loads of several samples in flight per thread
    const float* xb = xm + b0 * bstride;
    const int tot = (b1 - b0) * rowv;
    Walk3 wk(tid, W, Cv, 256);
#pragma unroll 4
    for (int e = tid; e < tot; e += 256, wk.next()) {
        float v[V];
        ldv<V>(xb + wk.r * bstride + (long long)wk.x * a.x_ps + wk.c * V, v);
#pragma unroll
        for (int j = 0; j < V; ++j) {
            s += (double)v[j];
            q += (double)v[j] * v[j];
        }
    }
    s = block_sum(s, red);
    q = block_sum(q, red);
    if (tid == 0) {
        double* o = part + (((long long)m * S + sl) * H + h) * 2;
        o[0] = s;
        o[1] = q;
    }
}

// The head site: z = ELU(x scale + shift) stored for the GAP (dn_bn_coef ran first)
__global__ __launch_bounds__(256) void dn_bn_apply_kernel(BnArgs a) {
    const int row = blockIdx.x, m = blockIdx.y, tid = threadIdx.x;
    const int H = a.H, W = a.W, Cin = a.Cin;
    const int b = row / H, h = row - b * H;
    const int rowe = W * Cin;
    const float* coef = a.coef + m * a.coef_ms;
    const float s = coef[2 * H + h], t = coef[3 * H + h];
    const float* xr = a.x + m * a.x_ms + ((long long)b * H + h) * W * a.x_ps;
    float* zr = a.z + m * a.z_ms + ((long long)b * H + h) * rowe;
    Walk2 wk(tid, Cin, 256);
    for (int e = tid; e < rowe; e += 256, wk.next()) {
        const int w = wk.q, c = wk.c;
        zr[e] = bn_elu(xr[(long long)w * a.x_ps + c], s, t);
    }
}

// The coefficients of a site: grid (member), one thread per image row h.  Training:
// the S slice partials folded in fixed order (plus, for an incremental site, the
// previous site's totals -- its statistics cover the channels before c0), stored
// as this site's totals, then the moving averages; evaluation: the moving
// averages.  Writes (mean, inv, scale = gamma inv, shift = beta - mean scale).
__global__ __launch_bounds__(64) void dn_bn_coef_kernel(BnArgs a, const double* __restrict__ part, int S) {
    const int m = blockIdx.x;
    const int H = a.H, rowe = a.W * a.Cin;
    for (int h = threadIdx.x; h < H; h += 64) {
        float mean, var;
        if (a.train) {
            double* tt = a.tot + ((long long)m * H + h) * 2;
            double s = a.prev ? tt[0] : 0.0, q = a.prev ? tt[1] : 0.0;
            for (int sl = 0; sl < S; ++sl) {
                const double* o = part + (((long long)m * S + sl) * H + h) * 2;
                s += o[0];
                q += o[1];
            }
            tt[0] = s;
            tt[1] = q;
            const double n = (double)a.B * rowe;
            const double mu = s / n;
            mean = (float)mu;
            var = (float)fmax(q / n - mu * mu, 0.0);
            float* st = a.state + m * a.s_ms;
            st[a.mm_off + h] = kBnMomentum * st[a.mm_off + h] + (1.f - kBnMomentum) * mean;
            st[a.mv_off + h] = kBnMomentum * st[a.mv_off + h] + (1.f - kBnMomentum) * var;
        } else {
            const float* st = a.state + m * a.s_ms;
            mean = st[a.mm_off + h];
            var = st[a.mv_off + h];
        }
        const float inv = (float)(1.0 / sqrt((double)var + (double)kBnEps));
        const float* pm = a.params + m * a.p_ms;
        const float gam = pm[a.g_off + h], bet = pm[a.b_off + h];
        float* coef = a.coef + m * a.coef_ms;
        coef[h] = mean;
        coef[H + h] = inv;
        coef[2 * H + h] = gam * inv;
        coef[3 * H + h] = bet - mean * gam * inv;
    }
}

// BN + ELU backward.  dy = dz * ELU'(z) (ELU' = 1 for z > 0, else z + 1);
// dbeta[h] = sum dy, dgamma[h] = sum dy xhat (dn_bn_bwd_reduce: slice partials,
// folded in fixed order by dn_bn_bwd_fold into slot 0, which also stores the
// gradients); dx = gamma inv / n (n dy - dbeta - xhat dgamma) stored or added
// into dcat (dn_bn_bwd_apply: two (b, h) rows per 256-thread block, no barrier).
// ELU'(y) from cat (z is never stored): 1 for y > 0, else e^y (= z + 1; the
// hardware exp is enough for a derivative factor and far cheaper than expm1f)
template <int V>
__device__ __forceinline__ void bn_dy(const BnArgs& a, const float (&x)[V], float s, float t, const float* dzr,
                                      const float* dgr, int e, int c, float (&dy)[V]) {
    float d[V];
    if (a.bcast) {
        ldv<V>(dgr + c * V, d);
#pragma unroll
        for (int j = 0; j < V; ++j) d[j] *= a.inv_hw;
    } else {
        ldv<V>(dzr + e * V, d);
    }
#pragma unroll
    for (int j = 0; j < V; ++j) {
        const float y = x[j] * s + t;
        dy[j] = d[j] * (y > 0.f ? 1.f : __expf(y));
    }
}

template <int V>
__global__ __launch_bounds__(256) void dn_bn_bwd_reduce_kernel(BnArgs a, double* __restrict__ part, int S, int bs) {
    __shared__ double red[4];
    const int h = blockIdx.x, sl = blockIdx.y, m = blockIdx.z, tid = threadIdx.x;
    const int H = a.H, W = a.W, Cin = a.Cin, Cv = Cin / V;
    const int rowe = W * Cin, rowv = W * Cv;
    const float* coef = a.coef + m * a.coef_ms;
    const float mean = coef[h], inv = coef[H + h], bs_ = coef[2 * H + h], bt_ = coef[3 * H + h];
    const int b0 = sl * bs, b1 = min(a.B, b0 + bs);
    double sdy = 0.0, sdyx = 0.0;
    const long long xbs = (long long)H * W * a.x_ps, zbs = (long long)H * rowe;
    const float* xb = a.x + m * a.x_ms + ((long long)b0 * H + h) * W * a.x_ps;
    const float* dzb = a.bcast ? nullptr : a.dz + m * a.dz_ms + ((long long)b0 * H + h) * rowe;
    const float* dgb = a.bcast ? a.dg + m * a.dg_ms + (long long)b0 * Cin : nullptr;
    const int tot = (b1 - b0) * rowv;
    Walk3 wk(tid, W, Cv, 256);   // (sample, pixel, channel group) flattened, as dn_bn_stats
#pragma unroll 2
    for (int e = tid; e < tot; e += 256, wk.next()) {
        float xv[V], dy[V];
        ldv<V>(xb + wk.r * xbs + (long long)wk.x * a.x_ps + wk.c * V, xv);
        bn_dy<V>(a, xv, bs_, bt_, a.bcast ? nullptr : dzb + wk.r * zbs, a.bcast ? dgb + wk.r * Cin : nullptr,
                 wk.x * Cv + wk.c, wk.c, dy);
#pragma unroll
        for (int j = 0; j < V; ++j) {
            const float xh = (xv[j] - mean) * inv;
            sdy += dy[j];
            sdyx += (double)dy[j] * xh;
        }
    }
    sdy = block_sum(sdy, red);
    sdyx = block_sum(sdyx, red);
    if (tid == 0) {
        double* o = part + (((long long)m * S + sl) * H + h) * 2;
        o[0] = sdy;
        o[1] = sdyx;
    }
}

// grid (member), one thread per image row h: the S slice partials summed in fixed
// order into slot 0 (each thread reads and writes only its own h), dgamma / dbeta
__global__ __launch_bounds__(64) void dn_bn_bwd_fold_kernel(BnArgs a, double* __restrict__ part, int S) {
    const int m = blockIdx.x, H = a.H;
    for (int h = threadIdx.x; h < H; h += 64) {
        double sdy = 0.0, sdyx = 0.0;
        for (int sl = 0; sl < S; ++sl) {
            const double* o = part + (((long long)m * S + sl) * H + h) * 2;
            sdy += o[0];
            sdyx += o[1];
        }
        double* o = part + ((long long)m * S * H + h) * 2;
        o[0] = sdy;
        o[1] = sdyx;
        float* gm = a.grads + m * a.p_ms;
        gm[a.g_off + h] = (float)sdyx;
        gm[a.b_off + h] = (float)sdy;
    }
}

// grid (H, member), one wave per image row: the fold for the epilogue-fused reduce's
// many slices (sample x row segment): lane l sums slices l, l + 64, ... in order, then a
// fixed butterfly; slot 0 and the gradients as dn_bn_bwd_fold
__global__ __launch_bounds__(64) void dn_bn_bwd_fold_wide_kernel(BnArgs a, double* __restrict__ part, int S) {
    const int h = blockIdx.x, m = blockIdx.y, H = a.H, lane = threadIdx.x;
    double sdy = 0.0, sdyx = 0.0;
    for (int sl = lane; sl < S; sl += 64) {
        const double* o = part + (((long long)m * S + sl) * H + h) * 2;
        sdy += o[0];
        sdyx += o[1];
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        sdy += __shfl_xor(sdy, off);
        sdyx += __shfl_xor(sdyx, off);
    }
    __syncthreads();   // every lane has read its slices before lane 0 overwrites slot 0 (slice 0)
    if (lane == 0) {
        double* o = part + ((long long)m * S * H + h) * 2;
        o[0] = sdy;
        o[1] = sdyx;
        float* gm = a.grads + m * a.p_ms;
        gm[a.g_off + h] = (float)sdyx;
        gm[a.b_off + h] = (float)sdy;
    }
}

template <int V>
__global__ __launch_bounds__(256) void dn_bn_bwd_apply_kernel(BnArgs a, const double* __restrict__ part, int S) {
    const int tid = threadIdx.x & 127, m = blockIdx.y;
    const int row = blockIdx.x * 2 + (threadIdx.x >> 7);
    const int H = a.H, W = a.W, Cin = a.Cin, Cv = Cin / V;
    if (row >= a.B * H) return;
    const int b = row / H, h = row - b * H;
    const int rowe = W * Cin, rowv = W * Cv;
    const float* coef = a.coef + m * a.coef_ms;
    const float mean = coef[h], inv = coef[H + h], bs_ = coef[2 * H + h], bt_ = coef[3 * H + h];
    const double* o = part + ((long long)m * S * H + h) * 2;   // folded: slot 0
    const float fb = (float)o[0], fg = (float)o[1];
    const float n = (float)a.B * rowe;
    const float ca = a.params[m * a.p_ms + a.g_off + h] * inv / n;
    const float* xr = a.x + m * a.x_ms + ((long long)b * H + h) * W * a.x_ps;
    const long long zo = ((long long)b * H + h) * rowe;
    const float* dzr = a.bcast ? nullptr : a.dz + m * a.dz_ms + zo;
    const float* dgr = a.bcast ? a.dg + m * a.dg_ms + (long long)b * Cin : nullptr;
    float* dxr = a.dx + m * a.dx_ms + ((long long)b * H + h) * W * a.dx_ps;
    Walk2 wk(tid, Cv, 128);
    for (int e = tid; e < rowv; e += 128, wk.next()) {
        float xv[V], dy[V], v[V];
        ldv<V>(xr + (long long)wk.q * a.x_ps + wk.c * V, xv);
        bn_dy<V>(a, xv, bs_, bt_, dzr, dgr, e, wk.c, dy);
#pragma unroll
        for (int j = 0; j < V; ++j) {
            const float xh = (xv[j] - mean) * inv;
            v[j] = ca * (n * dy[j] - fb - xh * fg);
        }
        float* q = dxr + (long long)wk.q * a.dx_ps + wk.c * V;
        if (a.accumulate) {
            float d[V];
            ldv<V>(q, d);
#pragma unroll
            for (int j = 0; j < V; ++j) v[j] += d[j];
        }
        stv<V>(q, v);
    }
}

// AvgPool2D((2,2), strides 2, valid): t [B][H][W][C] -> cat' [B][H/2][W/2][.] channels [0, C).
// Two output rows per 256-thread block (grid (ceil(B H/2 / 2), member)), each row
// walked as V-float channel groups -- no per-element 64-bit divisions.
template <int V>
__global__ __launch_bounds__(256) void dn_pool_fwd_kernel(const float* __restrict__ t, long long t_ms,
                                                          float* __restrict__ out, long long o_ms, int o_ps, int B,
                                                          int H, int W, int C) {
    const int m = blockIdx.y, H2 = H / 2, W2 = W / 2, Cv = C / V;
    const int row = blockIdx.x * 2 + (threadIdx.x >> 7), tid = threadIdx.x & 127;
    if (row >= B * H2) return;
    const int b = row / H2, y = row - b * H2;
    const float* tr = t + m * t_ms + ((long long)b * H + 2 * y) * W * C;
    float* orow = out + m * o_ms + (long long)row * W2 * o_ps;
    const long long WC = (long long)W * C;
    Walk2 wk(tid, Cv, 128);
    for (int e = tid; e < W2 * Cv; e += 128, wk.next()) {
        const float* s = tr + (long long)(2 * wk.q) * C + wk.c * V;
        float s0[V], s1[V], s2[V], s3[V], v[V];
        ldv<V>(s, s0);
        ldv<V>(s + C, s1);
        ldv<V>(s + WC, s2);
        ldv<V>(s + WC + C, s3);
#pragma unroll
        for (int j = 0; j < V; ++j) v[j] = 0.25f * (s0[j] + s1[j] + s2[j] + s3[j]);
        stv<V>(orow + (long long)wk.q * o_ps + wk.c * V, v);
    }
}

// dt [B][H][W][C] = dcat'[y/2][x/2][c] / 4 (zero in a floor-mode odd last row / column)
template <int V>
__global__ __launch_bounds__(256) void dn_pool_bwd_kernel(const float* __restrict__ dcat, long long d_ms, int d_ps,
                                                          float* __restrict__ dt, long long t_ms, int B, int H, int W,
                                                          int C) {
    const int m = blockIdx.y, H2 = H / 2, W2 = W / 2, Cv = C / V;
    const int row = blockIdx.x * 2 + (threadIdx.x >> 7), tid = threadIdx.x & 127;
    if (row >= B * H) return;
    const int b = row / H, y = row - b * H;
    const bool live_y = (y >> 1) < H2;
    const float* dr = dcat + m * d_ms + ((long long)b * H2 + (y >> 1)) * W2 * d_ps;
    float* trow = dt + m * t_ms + (long long)row * W * C;
    Walk2 wk(tid, Cv, 128);
    for (int e = tid; e < W * Cv; e += 128, wk.next()) {
        float v[V];
        if (live_y && (wk.q >> 1) < W2) {
            ldv<V>(dr + (long long)(wk.q >> 1) * d_ps + wk.c * V, v);
#pragma unroll
            for (int j = 0; j < V; ++j) v[j] *= 0.25f;
        } else {
#pragma unroll
            for (int j = 0; j < V; ++j) v[j] = 0.f;
        }
        stv<V>(trow + e * V, v);
    }
}

// ============================================================================
// Head: GlobalAveragePooling -> Dense(classes) -> softmax -> categorical CE.
// dn_head_fwd: one workgroup per (sample, member).  Writes g [B][C], per-sample CE,
// correct flag and dlogits = live * (p - onehot) / B (Keras: p /= sum p, clip to
// [1e-7, 1 - 1e-7]: a clipped target has zero gradient).
// ============================================================================
struct HeadArgs {
    const float* z; long long z_ms;
    const float* params; long long p_ms; long long wd_off, bd_off;
    float* grads;
    float* g; float* dl; float* ce; float* dg; long long h_ms;   // head scratch, member stride h_ms
    const int* labels; const int* order; long long ord_ms; long long row0;
    float* loss_out; float* loss_sum; int* correct;
    int B, HW, C, classes, train;
};

__global__ __launch_bounds__(256) void dn_head_fwd_kernel(HeadArgs a) {
    extern __shared__ __attribute__((aligned(16))) float hs[];
    const int b = blockIdx.x, m = blockIdx.y, tid = threadIdx.x;
    const int C = a.C, K = a.classes, HW = a.HW, B = a.B;
    float* g = hs;          // [C]
    float* lg = hs + C;     // [K]
    const float* zb = a.z + m * a.z_ms + (long long)b * HW * C;
    const float inv_hw = 1.f / HW;
    for (int c = tid; c < C; c += 256) {
        float s = 0.f;
        for (int p = 0; p < HW; ++p) s += zb[(long long)p * C + c];
        s *= inv_hw;
        g[c] = s;
        a.g[m * a.h_ms + (long long)b * C + c] = s;
    }
    __syncthreads();
    const float* pm = a.params + m * a.p_ms;
    for (int j = tid; j < K; j += 256) {
        float s = pm[a.bd_off + j];
        for (int c = 0; c < C; ++c) s += g[c] * pm[a.wd_off + (long long)c * K + j];
        lg[j] = s;
    }
    __syncthreads();
    if (tid == 0) {
        const int y = a.labels[a.order[m * a.ord_ms + a.row0 + b]];
        float mx = lg[0];
        int arg = 0;
        for (int j = 1; j < K; ++j)
            if (lg[j] > mx) { mx = lg[j]; arg = j; }
        float S = 0.f;
        for (int j = 0; j < K; ++j) { lg[j] = expf(lg[j] - mx); S += lg[j]; }
        float S2 = 0.f;
        for (int j = 0; j < K; ++j) { lg[j] /= S; S2 += lg[j]; }
        for (int j = 0; j < K; ++j) lg[j] /= S2;
        const float pt = lg[y];
        const float pc = fminf(fmaxf(pt, kCeEps), 1.f - kCeEps);
        float* hm = a.ce + m * a.h_ms;
        hm[b] = -logf(pc);
        hm[B + b] = arg == y ? 1.f : 0.f;
        const float live = (pt >= kCeEps && pt <= 1.f - kCeEps) ? 1.f : 0.f;
        float* dl = a.dl + m * a.h_ms + (long long)b * K;
        for (int j = 0; j < K; ++j) dl[j] = live * (lg[j] - (j == y ? 1.f : 0.f)) / B;
    }
}

// One workgroup per member.  Train: loss_out = mean CE + l2 penalty; dense grads;
// dg = dlogits . wd^T.  Eval: loss_sum += sum CE, correct += sum correct.
__global__ __launch_bounds__(256) void dn_head_reduce_kernel(HeadArgs a, long long n_params) {
    __shared__ double red[4];
    const int m = blockIdx.x, tid = threadIdx.x;
    const int C = a.C, K = a.classes, B = a.B;
    const float* hm = a.ce + m * a.h_ms;
    double s = 0.0, cor = 0.0;
    for (int b = tid; b < B; b += 256) { s += hm[b]; cor += hm[B + b]; }
    const double ce_sum = block_sum(s, red);
    const double cor_sum = block_sum(cor, red);
    if (!a.train) {
        if (tid == 0) {
            a.loss_sum[m] += (float)ce_sum;
            a.correct[m] += (int)(cor_sum + 0.5);
        }
        return;
    }
    const float* pm = a.params + m * a.p_ms;
    double pen = 0.0;
    for (long long i = tid; i < n_params; i += 256) pen += (double)pm[i] * pm[i];
    pen = block_sum(pen, red);
    if (tid == 0) a.loss_out[m] = (float)(ce_sum / B + (double)kL2 * pen);
    const float* g = a.g + m * a.h_ms;
    const float* dl = a.dl + m * a.h_ms;
    float* gm = a.grads + m * a.p_ms;
    for (int e = tid; e < C * K; e += 256) {
        const int c = e / K, j = e - c * K;
        float v = 0.f;
        for (int b = 0; b < B; ++b) v += g[(long long)b * C + c] * dl[(long long)b * K + j];
        gm[a.wd_off + e] = v;
    }
    for (int j = tid; j < K; j += 256) {
        float v = 0.f;
        for (int b = 0; b < B; ++b) v += dl[(long long)b * K + j];
        gm[a.bd_off + j] = v;
    }
    float* dg = a.dg + m * a.h_ms;
    for (int e = tid; e < B * C; e += 256) {
        const int b = e / C, c = e - b * C;
        float v = 0.f;
        for (int j = 0; j < K; ++j) v += dl[(long long)b * K + j] * pm[a.wd_off + (long long)c * K + j];
        dg[e] = v;
    }
}

// Per-member l2 penalty 1e-4 * sum w^2 (Keras adds it to loss and val_loss).
__global__ __launch_bounds__(256) void dn_penalty_kernel(const float* __restrict__ params, long long p_ms, long long n,
                                                         float* __restrict__ out) {
    __shared__ double red[4];
    const float* pm = params + blockIdx.x * p_ms;
    double s = 0.0;
    for (long long i = threadIdx.x; i < n; i += 256) s += (double)pm[i] * pm[i];
    s = block_sum(s, red);
    if (threadIdx.x == 0) out[blockIdx.x] = (float)((double)kL2 * s);
}

// Keras Adam with the l2(1e-4) gradient 2e-4 w folded in (every DenseNet tensor is
// regularised: conv kernels, gamma/beta, dense kernel + bias -- densenet.py:24-33, 188-191).
__global__ void dn_adam_kernel(float* __restrict__ params, float* __restrict__ grads, float* __restrict__ mo,
                               float* __restrict__ vo, long long p_ms, long long n, const float* __restrict__ lr, int t) {
    const int m = blockIdx.y;
    const float b1 = 0.9f, b2 = 0.999f, eps = 1e-8f;
    const double corr = sqrt(1.0 - pow((double)b2, t)) / (1.0 - pow((double)b1, t));
    const float lr_t = (float)(lr[m] * corr);
    const long long base = m * p_ms;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        const float w = params[base + i];
        const float g = grads[base + i] + 2.f * kL2 * w;
        const float mm = b1 * mo[base + i] + (1.f - b1) * g;
        const float vv = b2 * vo[base + i] + (1.f - b2) * g * g;
        mo[base + i] = mm;
        vo[base + i] = vv;
        params[base + i] = w - lr_t * mm / (sqrtf(vv) + eps);
    }
}

// ============================================================================
// Host plan
// ============================================================================
enum Kind { K_CONV0 = 0, K_DENSE = 1, K_TRANS = 2, K_HEAD = 3 };

struct Layer {
    int kind, stage, H, W, cin, cout, ks, coff;
    long long w_off = -1, g_off = -1, b_off = -1, mm_off = -1, mv_off = -1;   // params / state
    long long wf_off = -1, wd_off_act = -1;    // padded fwd / dgrad weights (act arena)
    int wf_rows = 0, wf_n16 = 0, wd_rows = 0, wd_n16 = 0;
    long long z_off = -1, t_off = -1, coef_off = -1;
    int G = 1, spg = 1, R = 1, Rw = 1;
    int kw = 1;    // dn_wgrad3 k groups per workgroup (wg3_kw)
};

struct DnPlan {
    MpoDnArch arch{};
    int n = 0, B = 0;
    std::vector<Layer> layers;
    std::vector<int> sH, sW, sC;
    std::vector<long long> cat_off, dcat_off, cat_sz;
    long long n_params = 0, n_state = 0, act_floats = 0;
    long long wd_off = 0, bd_off = 0;
    // member strides of the activation buffers (floats)
    std::vector<long long> cat_ms;
    long long z_ms_max = 0;
    long long dz_off = 0, dz_ms = 0, dt_off = 0, dt_ms = 0, part_off = 0, part_ms = 0, part2_off = 0, part2_ms = 0;
    long long part3_off = 0, part3_ms = 0;
    long long head_off = 0, head_ms = 0, lr_off = 0;
    long long bnp_off = 0;
    long long bnt_off = 0;      // fp64 BN totals of the latest site [n][H][2]      // fp64 BN slice partials [n][S][H][2] (shared by all sites)
    std::vector<int> bn_S, bn_bs;   // per layer: batch slices and samples per slice
    std::vector<int> bn_fS;         // per dense layer: the slices of its epilogue-fused BN backward reduce (0: none)
    bool bnfuse = true;             // MPO_DN_PLAN=bnfuse=0: dn_bn_bwd_reduce as its own pass
    float *params = nullptr, *grads = nullptr, *m = nullptr, *v = nullptr, *state = nullptr, *act = nullptr;
    bool bound = false;
    // the weight gradients (+ their slab reduction) of the backward run on a second
    // stream beside the input-gradient convs and BN backward (MPO_DN_PLAN=streams=1:
    // one stream); see enqueue_backward for what they read and write
    mpo::SideStream side;
    // r06: a second weight-gradient stream (pooled slot 1): the layers' weight gradients
    // alternate between the two, each pair of streams with its own slab buffer
    // (MPO_DN_PLAN=wg2=0: one weight-gradient stream)
    mpo::SideStream side2, side3;
    bool wg2 = true;
    int wgs = 2;   // weight-gradient streams (MPO_DN_PLAN=wgs=3: a third, pooled slot 2)
    // the transitions' 1x1 convs streamed by dn_conv1x1_kernel (MPO_DN_PLAN=c1x1=0: dn_conv_kernel)
    bool conv1x1 = true;
};

// (member stride, offset) allocator over the member-major activation arena
struct Arena {
    long long used = 0;
    int n;
    explicit Arena(int n_) : n(n_) {}
    // returns the offset; the per-member stride is the aligned size
    long long take(long long per_member, long long* ms) {
        const long long s = (per_member + 63) & ~63LL;
        const long long off = used;
        used += s * n;
        *ms = s;
        return off;
    }
};

// Choose rows per chunk so that R * W <= kMaxPix pixels.
int rows_per_chunk(int H, int W) { return std::max(1, std::min(H, kMaxPix / std::max(1, W))); }

// dn_conv's pooled epilogue: the chunk's m-tiles of outputs, NT 16 + 4 floats apart
// the population the work splits are sized for (build_plan): the reference search's
// 32 DenseNet trials per GPU
constexpr int kNominalMembers = 32;
constexpr int kWgTarget = 2048;   // weight-gradient workgroups per launch at kNominalMembers

size_t pool_tile_lds(int R, int W, int nt) { return (size_t)r16(R * W) * (nt * 16 + 4) * sizeof(float); }

size_t conv_lds(int R, int W, int ks, int cin) {
    const int img = (R + ks - 1) * (W + ks - 1) * conv_cp(cin);
    return (size_t)(r4(img) + r16(ks * ks * r4(cin)) + kKoffSlack) * sizeof(float);
}

// dn_wgrad3's k groups: the fewest m-waves mw (8 / kw) that keep every wave's
// m-tiles <= kWgMT; layers past one m-group keep mw = 8
int wg3_kw(int Kw) {
    const int mt = std::min(kWgRows / 16, (Kw + 15) / 16);
    int mw = 1;
    while (mw < kWgWaves && (mt + mw - 1) / mw > kWgMT) mw *= 2;
    return kWgWaves / mw;
}

size_t wg_lds(int R, int W, int ks, int cin, int nt, int kw) {
    if (ks == 1) return 0;   // dn_wgrad1: static LDS only
    const int img = (R + ks - 1) * (W + ks - 1) * wg_cp(cin);
    const int np = 4 * (((R * W + 3) >> 2) + kWgWaves);
    // k-group sums: the accumulators of the kq > 0 waves
    const size_t red = kw > 1 ? (size_t)(kWgWaves - kWgWaves / kw) * wg3_tpw(9 * cin, kWgWaves / kw) * nt * 256 : 0;
    return std::max((size_t)(r4(img) + np * wg_ns(nt) + np), red) * sizeof(float);
}

int build_plan(DnPlan& p) {
    const MpoDnArch& A = p.arch;
    const int L = (A.depth - 4) / 3;
    int H = A.H, W = A.W, f = A.nb_filter, stage = 0;
    auto& ls = p.layers;
    ls.push_back(Layer{K_CONV0, 0, H, W, A.C, f, 3, 0});
    for (int blk = 0; blk < A.nb_dense_block; ++blk) {
        for (int l = 0; l < L; ++l) {
            ls.push_back(Layer{K_DENSE, stage, H, W, f, A.growth, 3, f});
            f += A.growth;
        }
        if (blk < A.nb_dense_block - 1) {
            ls.push_back(Layer{K_TRANS, stage, H, W, f, f, 1, 0});
            p.sH.push_back(H); p.sW.push_back(W); p.sC.push_back(f);
            H /= 2; W /= 2;
            ++stage;
        }
    }
    ls.push_back(Layer{K_HEAD, stage, H, W, f, A.classes, 0, 0});
    p.sH.push_back(H); p.sW.push_back(W); p.sC.push_back(f);
    for (auto& ly : ls)
        if (ly.H < 1 || ly.W < 1 || ly.W > kMaxPix) return MPO_ENOTSUP;
    if (f > 1024 || A.classes > 1024) return MPO_ENOTSUP;

    // parameters (Keras creation order), 16-float aligned; moving stats
    long long po = 0, so = 0;
    auto take = [](long long& o, long long cnt) { const long long r = o; o += (cnt + 15) & ~15LL; return r; };
    for (auto& ly : ls) {
        if (ly.kind == K_CONV0) {
            ly.w_off = take(po, 9LL * ly.cin * ly.cout);
        } else if (ly.kind == K_HEAD) {
            ly.g_off = take(po, ly.H);
            ly.b_off = take(po, ly.H);
            p.wd_off = take(po, (long long)ly.cin * ly.cout);
            p.bd_off = take(po, ly.cout);
            ly.mm_off = take(so, ly.H);
            ly.mv_off = take(so, ly.H);
        } else {
            ly.g_off = take(po, ly.H);
            ly.b_off = take(po, ly.H);
            ly.w_off = take(po, (long long)ly.ks * ly.ks * ly.cin * ly.cout);
            ly.mm_off = take(so, ly.H);
            ly.mv_off = take(so, ly.H);
        }
    }
    p.n_params = (po + 63) & ~63LL;
    p.n_state = (so + 63) & ~63LL;

    // activation arena
    Arena ar(p.n);
    const int B = p.B;
    const int S = (int)p.sH.size();
    p.cat_off.resize(S); p.dcat_off.resize(S); p.cat_ms.resize(S);
    for (int s = 0; s < S; ++s) {
        const long long sz = (long long)B * p.sH[s] * p.sW[s] * p.sC[s];
        long long ms;
        p.cat_off[s] = ar.take(sz, &ms);
        p.dcat_off[s] = ar.take(sz, &ms);
        p.cat_ms[s] = ms;
    }
    long long dz_max = 0, dt_max = 0, part_max = 0;
    // The work splits (weight-gradient sample groups, BN batch slices) are sized for
    // a nominal population, never the actual one: they fix the order of the
    // partial sums, so a member's arithmetic must not depend on how many members
    // train beside it (tests/test_densenet_gpu.py::test_member_isolation_*).
    const int target = kWgTarget;
    for (auto& ly : ls) {
        long long ms;
        if (ly.kind != K_CONV0) {
            // z = ELU(BN(cat)) is stored for the head's GAP only; the other sites'
            // convs, weight gradients and BN backward form it from cat on the fly
            if (ly.kind == K_HEAD) ly.z_off = ar.take((long long)B * ly.H * ly.W * ly.cin, &ms);
            ly.coef_off = ar.take(4LL * ly.H, &ms);
            dz_max = std::max(dz_max, (long long)B * ly.H * ly.W * ly.cin);
        }
        if (ly.kind == K_TRANS) {
            ly.t_off = ar.take((long long)B * ly.H * ly.W * ly.cout, &ms);
            dt_max = std::max(dt_max, (long long)B * ly.H * ly.W * ly.cout);
        }
        if (ly.kind != K_HEAD) {
            const int taps = ly.ks * ly.ks;
            ly.wf_n16 = r16(ly.cout);
            ly.wf_rows = r16(taps * r4(ly.cin)) + kWRowsSlack;
            ly.wf_off = ar.take((long long)ly.wf_rows * ly.wf_n16, &ms);
            if (ly.kind != K_CONV0) {
                ly.wd_n16 = r16(ly.cin);
                ly.wd_rows = r16(taps * r4(ly.cout)) + kWRowsSlack;
                ly.wd_off_act = ar.take((long long)ly.wd_rows * ly.wd_n16, &ms);
            }
            ly.R = rows_per_chunk(ly.H, ly.W);
            ly.Rw = ly.R;
            const long long Kw = (long long)taps * ly.cin;
            const int mgroups = ly.ks == 1 ? 1 : (int)((Kw + kWgRows - 1) / kWgRows);
            const int gt = std::max(1, (target + mgroups * kNominalMembers - 1) / (mgroups * kNominalMembers));
            const int G0 = std::min(B, gt);
            ly.spg = (B + G0 - 1) / G0;
            ly.G = (B + ly.spg - 1) / ly.spg;
            ly.kw = ly.ks == 3 ? wg3_kw((int)Kw) : 1;
            part_max = std::max(part_max, (long long)ly.G * Kw * ly.cout);
        }
    }
    // BN batch slices: enough (h, slice, member) workgroups to fill the chip
    long long bnp_max = 0;
    p.bn_S.assign(ls.size(), 1);
    p.bn_bs.assign(ls.size(), B);
    for (size_t i = 0; i < ls.size(); ++i) {
        const Layer& ly = ls[i];
        if (ly.kind == K_CONV0) continue;
        const int want = std::max(1, (2048 + ly.H * kNominalMembers - 1) / (ly.H * kNominalMembers));
        const int bs = (B + std::min(B, want) - 1) / std::min(B, want);
        p.bn_bs[i] = bs;
        p.bn_S[i] = (B + bs - 1) / bs;
        bnp_max = std::max(bnp_max, (long long)p.bn_S[i] * ly.H * 2);
    }
    // the dense layers' BN backward reduce in their input-gradient conv's epilogue: one
    // partial per (sample, 16-pixel row segment) slice
    p.bn_fS.assign(ls.size(), 0);
    for (size_t i = 0; i < ls.size(); ++i) {
        const Layer& ly = ls[i];
        if (!p.bnfuse || ly.kind != K_DENSE || ly.ks != 3 || ly.W % 4 != 0 || (ly.W < 16 && 16 % ly.W != 0)) continue;
        p.bn_fS[i] = B * std::max(1, ly.W / 16);
        bnp_max = std::max(bnp_max, (long long)p.bn_fS[i] * ly.H * 2);
    }
    long long bnp_ms;
    p.bnp_off = ar.take(bnp_max * 2, &bnp_ms);   // doubles = 2 floats (arena offsets are 64-float aligned)
    int hmax = 1;
    for (const Layer& ly : ls) hmax = std::max(hmax, ly.H);
    long long bnt_ms;
    p.bnt_off = ar.take(4LL * hmax, &bnt_ms);     // [n][H][2] doubles, indexed contiguously
    p.dz_off = ar.take(dz_max, &p.dz_ms);
    p.dt_off = ar.take(std::max(dt_max, 1LL), &p.dt_ms);
    p.part_off = ar.take(part_max, &p.part_ms);
    if (p.wg2) p.part2_off = ar.take(part_max, &p.part2_ms);
    if (p.wg2 && p.wgs >= 3) p.part3_off = ar.take(part_max, &p.part3_ms);
    const Layer& hd = ls.back();
    // head scratch: g [B][C] | dl [B][K] | ce [2B] | dg [B][C]
    p.head_off = ar.take((long long)B * hd.cin * 2 + (long long)B * hd.cout + 2LL * B, &p.head_ms);
    p.lr_off = ar.used;   // per-member learning rates
    ar.used += (p.n + 63) & ~63LL;
    p.act_floats = ar.used;
    return MPO_OK;
}

template <int KS, int NT>
void launch_conv_t(const ConvArgs& a, dim3 grid, size_t lds, hipStream_t s) {
    auto kern = dn_conv_kernel<KS, NT>;
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(kern, grid, dim3(256), lds, s, a);
}

template <int NT>
void launch_wg3_t(const WgArgs& a, dim3 grid, size_t lds, hipStream_t s) {
    auto kern = dn_wgrad3_kernel<NT>;
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(kern, grid, dim3(kWgWaves * 64), lds, s, a);
}

// dn_conv1x1_kernel: a 2 x 8 patch per wave (even H, W % 8 == 0), float4 channel
// blocks (cin % 4 == 0, 16-B aligned rows), cin <= 16 CB with CB <= 4, N <= 64
bool conv1x1_ok(const ConvArgs& a) {
    auto al = [](const void* q) { return ((uintptr_t)q & 15) == 0; };
    return !a.order && a.H % 2 == 0 && a.W % 8 == 0 && a.Cin % 4 == 0 && a.Cin <= 64 && a.N <= 64 &&
           a.in_ps % 4 == 0 && a.in_ms % 4 == 0 && al(a.in);
}

template <int NT, int CB>
void launch_c1x1(const ConvArgs& a, dim3 grid, hipStream_t s) {
    if (a.pool) hipLaunchKernelGGL((dn_conv1x1_kernel<NT, CB, true>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((dn_conv1x1_kernel<NT, CB, false>), grid, dim3(256), 0, s, a);
}

template <int NT>
void launch_c1x1_cb(const ConvArgs& a, dim3 grid, int cb, hipStream_t s) {
    switch (cb) {
        case 1: launch_c1x1<NT, 1>(a, grid, s); break;
        case 2: launch_c1x1<NT, 2>(a, grid, s); break;
        case 3: launch_c1x1<NT, 3>(a, grid, s); break;
        default: launch_c1x1<NT, 4>(a, grid, s); break;
    }
}

int launch_conv1x1(const ConvArgs& a, int n_members, int B, hipStream_t s) {
    const int tiles = (a.H / 2) * (a.W / 8);
    const dim3 grid((tiles + 3) / 4, B, n_members);
    const int cb = (a.Cin + 15) / 16;
    switch ((a.N + 15) / 16) {
        case 1: launch_c1x1_cb<1>(a, grid, cb, s); break;
        case 2: launch_c1x1_cb<2>(a, grid, cb, s); break;
        case 3: launch_c1x1_cb<3>(a, grid, cb, s); break;
        default: launch_c1x1_cb<4>(a, grid, cb, s); break;
    }
    MPO_LAUNCH_CHECK();
    return MPO_OK;
}

template <int KS>
int launch_conv(const ConvArgs& a, int n_members, int B, hipStream_t s) {
    if (KS == 1 && a.c1x1 && conv1x1_ok(a)) return launch_conv1x1(a, n_members, B, s);
    const int nt = (a.N + 15) / 16;
    const dim3 grid((a.H + a.R - 1) / a.R, B, n_members);
    size_t lds = conv_lds(a.R, a.W, KS, a.Cin);
    if (a.pool) lds = std::max(lds, pool_tile_lds(a.R, a.W, nt));
    if (lds > ((size_t)160 << 10)) { mpo::set_error("dn_conv: LDS %zu B exceeds 160 KiB", lds); return MPO_ENOTSUP; }
    switch (nt) {
        case 1: launch_conv_t<KS, 1>(a, grid, lds, s); break;
        case 2: launch_conv_t<KS, 2>(a, grid, lds, s); break;
        case 3: launch_conv_t<KS, 3>(a, grid, lds, s); break;
        case 4: launch_conv_t<KS, 4>(a, grid, lds, s); break;
        case 5: launch_conv_t<KS, 5>(a, grid, lds, s); break;
        case 6: launch_conv_t<KS, 6>(a, grid, lds, s); break;
        default: mpo::set_error("dn_conv: %d output channels unsupported (max 96)", a.N); return MPO_ENOTSUP;
    }
    return MPO_OK;
}

// 1x1 weight gradient: MT x NT tiles per wave (<= 6 x 6, i.e. cin, cout <= 96)
template <int MT>
void launch_wg1_mt(const WgArgs& a, dim3 grid, int nt, hipStream_t s) {
    switch (nt) {
        case 1: hipLaunchKernelGGL((dn_wgrad1_kernel<MT, 1>), grid, dim3(kWgWaves * 64), 0, s, a); break;
        case 2: hipLaunchKernelGGL((dn_wgrad1_kernel<MT, 2>), grid, dim3(kWgWaves * 64), 0, s, a); break;
        case 3: hipLaunchKernelGGL((dn_wgrad1_kernel<MT, 3>), grid, dim3(kWgWaves * 64), 0, s, a); break;
        case 4: hipLaunchKernelGGL((dn_wgrad1_kernel<MT, 4>), grid, dim3(kWgWaves * 64), 0, s, a); break;
        default: break;
    }
}

int launch_wgrad(const WgArgs& a, int ks, int n_members, int G, hipStream_t s) {
    const int nt = (a.N + 15) / 16;
    if (ks == 1) {
        const int mt = (a.Cin + 15) / 16;
        if (mt > 4 || nt > 4) { mpo::set_error("dn_wgrad1: cin %d / cout %d > 64 unsupported", a.Cin, a.N); return MPO_ENOTSUP; }
        if (a.H > kWg1MaxH) { mpo::set_error("dn_wgrad1: %d image rows > %d unsupported", a.H, kWg1MaxH); return MPO_ENOTSUP; }
        const dim3 grid(1, G, n_members);
        switch (mt) {
            case 1: launch_wg1_mt<1>(a, grid, nt, s); break;
            case 2: launch_wg1_mt<2>(a, grid, nt, s); break;
            case 3: launch_wg1_mt<3>(a, grid, nt, s); break;
            case 4: launch_wg1_mt<4>(a, grid, nt, s); break;
            default: break;
        }
        return MPO_OK;
    }
    const int Kw = 9 * a.Cin;
    const dim3 grid((Kw + kWgRows - 1) / kWgRows, G, n_members);
    const size_t lds = wg_lds(a.R, a.W, 3, a.Cin, nt, a.kw);
    if (lds > ((size_t)160 << 10)) { mpo::set_error("dn_wgrad: LDS %zu B exceeds 160 KiB", lds); return MPO_ENOTSUP; }
    switch (nt) {
        case 1: launch_wg3_t<1>(a, grid, lds, s); break;
        case 2: launch_wg3_t<2>(a, grid, lds, s); break;
        case 3: launch_wg3_t<3>(a, grid, lds, s); break;
        case 4: launch_wg3_t<4>(a, grid, lds, s); break;
        default: mpo::set_error("dn_wgrad: %d output channels unsupported (max 64)", a.N); return MPO_ENOTSUP;
    }
    return MPO_OK;
}

inline dim3 flat_grid(long long total, int n_members) {
    long long bx = (total + 255) / 256;
    bx = std::max(1LL, std::min(bx, 1024LL));
    return dim3((unsigned)bx, n_members);
}

#define DN_TRY(x)                     \
    do {                              \
        const int rc_ = (x);          \
        if (rc_ != MPO_OK) return rc_; \
    } while (0)

int enqueue_prep(DnPlan& p, bool with_dgrad, hipStream_t s) {
    for (auto& ly : p.layers) {
        if (ly.kind == K_HEAD) continue;
        const int taps = ly.ks * ly.ks;
        const long long wms = (long long)ly.wf_rows * ly.wf_n16;
        hipLaunchKernelGGL(dn_prep_kernel, flat_grid(wms, p.n), dim3(256), 0, s, p.params, p.n_params, ly.w_off,
                           p.act + ly.wf_off, ((wms + 63) & ~63LL), taps, ly.cin, ly.cout, ly.wf_rows, ly.wf_n16, 0);
        if (with_dgrad && ly.kind != K_CONV0) {
            const long long dms = (long long)ly.wd_rows * ly.wd_n16;
            hipLaunchKernelGGL(dn_prep_kernel, flat_grid(dms, p.n), dim3(256), 0, s, p.params, p.n_params, ly.w_off,
                               p.act + ly.wd_off_act, ((dms + 63) & ~63LL), taps, ly.cin, ly.cout, ly.wd_rows,
                               ly.wd_n16, 1);
        }
    }
    MPO_LAUNCH_CHECK();
    return MPO_OK;
}

// float4 rows for the BN kernels: channel count, pixel strides, member strides and
// base pointers all multiples of 4 floats (every reference geometry; an odd growth
// rate falls back to the scalar instances)
bool bn_vec4(const BnArgs& a) {
    auto al = [](const void* q) { return ((uintptr_t)q & 15) == 0; };
    bool ok = a.Cin % 4 == 0 && a.c0 % 4 == 0 && a.x_ps % 4 == 0 && a.x_ms % 4 == 0 && al(a.x);
    ok = ok && a.dx_ps % 4 == 0 && a.dx_ms % 4 == 0 && al(a.dx);
    ok = ok && (a.bcast ? a.dg_ms % 4 == 0 && al(a.dg) : a.dz_ms % 4 == 0 && al(a.dz));
    return ok;
}

bool pool_vec4(int C, int ps, long long ms_a, long long ms_b, const float* pa, const float* pb) {
    auto al = [](const void* q) { return ((uintptr_t)q & 15) == 0; };
    return C % 4 == 0 && ps % 4 == 0 && ms_a % 4 == 0 && ms_b % 4 == 0 && al(pa) && al(pb);
}

BnArgs bn_args(DnPlan& p, const Layer& ly, bool train) {
    BnArgs a{};
    const int s = ly.stage;
    a.x = p.act + p.cat_off[s]; a.x_ms = p.cat_ms[s]; a.x_ps = p.sC[s];
    a.z = ly.z_off >= 0 ? p.act + ly.z_off : nullptr;
    a.z_ms = ((long long)p.B * ly.H * ly.W * ly.cin + 63) & ~63LL;
    a.coef = p.act + ly.coef_off; a.coef_ms = (4LL * ly.H + 63) & ~63LL;
    a.params = p.params; a.p_ms = p.n_params; a.g_off = ly.g_off; a.b_off = ly.b_off;
    a.state = p.state; a.s_ms = p.n_state; a.mm_off = ly.mm_off; a.mv_off = ly.mv_off;
    a.grads = p.grads;
    a.tot = reinterpret_cast<double*>(p.act + p.bnt_off);
    a.B = p.B; a.H = ly.H; a.W = ly.W; a.Cin = ly.cin; a.train = train ? 1 : 0;
    return a;
}

HeadArgs head_args(DnPlan& p, const int* labels, const int* order, long long ord_ms, long long row0, bool train) {
    const Layer& hd = p.layers.back();
    HeadArgs h{};
    h.z = p.act + hd.z_off; h.z_ms = ((long long)p.B * hd.H * hd.W * hd.cin + 63) & ~63LL;
    h.params = p.params; h.p_ms = p.n_params; h.wd_off = p.wd_off; h.bd_off = p.bd_off;
    h.grads = p.grads;
    float* base = p.act + p.head_off;
    const long long BC = (long long)p.B * hd.cin, BK = (long long)p.B * hd.cout;
    h.g = base; h.dl = base + BC; h.ce = base + BC + BK; h.dg = base + BC + BK + 2LL * p.B; h.h_ms = p.head_ms;
    h.labels = labels; h.order = order; h.ord_ms = ord_ms; h.row0 = row0;
    h.B = p.B; h.HW = hd.H * hd.W; h.C = hd.cin; h.classes = hd.cout; h.train = train ? 1 : 0;
    return h;
}

int enqueue_forward(DnPlan& p, const float* x, const int* labels, const int* order, long long ord_ms, long long row0,
                    bool train, float* loss_out, float* loss_sum, int* correct, hipStream_t s) {
    const int B = p.B, n = p.n;
    for (auto& ly : p.layers) {
        const int st = ly.stage;
        if (ly.kind == K_CONV0) {
            ConvArgs c{};
            c.in = x; c.in_ps = ly.cin; c.order = order; c.ord_ms = ord_ms; c.row0 = row0;
            c.img_floats = (long long)ly.H * ly.W * ly.cin;
            c.w = p.act + ly.wf_off; c.w_ms = ((long long)ly.wf_rows * ly.wf_n16 + 63) & ~63LL;
            c.out = p.act + p.cat_off[0]; c.out_ms = p.cat_ms[0]; c.out_ps = p.sC[0];
            c.H = ly.H; c.W = ly.W; c.Cin = ly.cin; c.N = ly.cout; c.R = ly.R;
            DN_TRY(launch_conv<3>(c, n, B, s));
            continue;
        }
        BnArgs bn = bn_args(p, ly, train);
        const size_t li = &ly - p.layers.data();
        double* bnp = reinterpret_cast<double*>(p.act + p.bnp_off);
        // a dense layer's or transition's input is the previous dense layer's input plus
        // that layer's growth slice: only the slice is read, its totals carried over
        const Layer* pv = li > 0 ? &p.layers[li - 1] : nullptr;
        if (pv && pv->kind == K_DENSE && pv->stage == ly.stage && pv->coff == pv->cin &&
            pv->cin + pv->cout == ly.cin) {
            bn.c0 = pv->cin;
            bn.prev = 1;
        }
        if (train) {
            auto kern = bn_vec4(bn) ? dn_bn_stats_kernel<4> : dn_bn_stats_kernel<1>;
            hipLaunchKernelGGL(kern, dim3(ly.H, p.bn_S[li], n), dim3(256), 0, s, bn, bnp, p.bn_S[li], p.bn_bs[li]);
        }
        hipLaunchKernelGGL(dn_bn_coef_kernel, dim3(n), dim3(64), 0, s, bn, (const double*)bnp, p.bn_S[li]);
        if (ly.kind == K_HEAD)   // the head's GAP reads z: the only site that stores it
            hipLaunchKernelGGL(dn_bn_apply_kernel, dim3(B * ly.H, n), dim3(256), 0, s, bn);
        if (ly.kind == K_HEAD) {
            HeadArgs h = head_args(p, labels, order, ord_ms, row0, train);
            h.loss_out = loss_out; h.loss_sum = loss_sum; h.correct = correct;
            const size_t lds = (size_t)(h.C + h.classes) * sizeof(float);
            hipLaunchKernelGGL(dn_head_fwd_kernel, dim3(B, n), dim3(256), lds, s, h);
            hipLaunchKernelGGL(dn_head_reduce_kernel, dim3(n), dim3(256), 0, s, h, p.n_params);
            continue;
        }
        ConvArgs c{};
        c.in = bn.x; c.in_ms = bn.x_ms; c.in_ps = bn.x_ps;   // cat: the conv stages ELU(BN(x))
        c.bnc = bn.coef; c.bnc_ms = bn.coef_ms;
        c.w = p.act + ly.wf_off; c.w_ms = ((long long)ly.wf_rows * ly.wf_n16 + 63) & ~63LL;
        c.H = ly.H; c.W = ly.W; c.Cin = ly.cin; c.N = ly.cout; c.R = ly.R;
        c.c1x1 = p.conv1x1 ? 1 : 0;
        if (ly.kind == K_DENSE) {
            c.out = p.act + p.cat_off[st] + ly.coff; c.out_ms = p.cat_ms[st]; c.out_ps = p.sC[st];
            DN_TRY(launch_conv<3>(c, n, B, s));
        } else {
            if (ly.R % 2 == 0 || (c.c1x1 && conv1x1_ok(c))) {
                // AvgPool2 in the conv's epilogue: straight into the next stage's concat
                c.out = p.act + p.cat_off[st + 1]; c.out_ms = p.cat_ms[st + 1]; c.out_ps = p.sC[st + 1];
                c.pool = 1;
                DN_TRY(launch_conv<1>(c, n, B, s));
                continue;
            }
            const long long tms = ((long long)B * ly.H * ly.W * ly.cout + 63) & ~63LL;
            c.out = p.act + ly.t_off; c.out_ms = tms; c.out_ps = ly.cout;
            DN_TRY(launch_conv<1>(c, n, B, s));
            const bool v4 = pool_vec4(ly.cout, p.sC[st + 1], tms, p.cat_ms[st + 1], p.act + ly.t_off,
                                      p.act + p.cat_off[st + 1]);
            hipLaunchKernelGGL(v4 ? dn_pool_fwd_kernel<4> : dn_pool_fwd_kernel<1>,
                               dim3((B * (ly.H / 2) + 1) / 2, n), dim3(256), 0, s, p.act + ly.t_off, tms,
                               p.act + p.cat_off[st + 1], p.cat_ms[st + 1], p.sC[st + 1], B, ly.H, ly.W, ly.cout);
        }
    }
    MPO_LAUNCH_CHECK();
    return MPO_OK;
}

void enqueue_bn_bwd(DnPlan& p, const BnArgs& bn, int li, hipStream_t s, int fused_S = 0) {
    double* bnp = reinterpret_cast<double*>(p.act + p.bnp_off);
    const int S = fused_S > 0 ? fused_S : p.bn_S[li];
    const bool v4 = bn_vec4(bn);
    if (fused_S <= 0)   // else the input-gradient conv's epilogue wrote the slice partials
        hipLaunchKernelGGL(v4 ? dn_bn_bwd_reduce_kernel<4> : dn_bn_bwd_reduce_kernel<1>, dim3(bn.H, S, p.n),
                           dim3(256), 0, s, bn, bnp, S, p.bn_bs[li]);
    if (fused_S > 0) hipLaunchKernelGGL(dn_bn_bwd_fold_wide_kernel, dim3(bn.H, p.n), dim3(64), 0, s, bn, bnp, S);
    else hipLaunchKernelGGL(dn_bn_bwd_fold_kernel, dim3(p.n), dim3(64), 0, s, bn, bnp, S);
    hipLaunchKernelGGL(v4 ? dn_bn_bwd_apply_kernel<4> : dn_bn_bwd_apply_kernel<1>, dim3((p.B * bn.H + 1) / 2, p.n),
                       dim3(256), 0, s, bn, (const double*)bnp, S);
}

int enqueue_backward(DnPlan& p, const float* x, const int* order, long long ord_ms, long long row0, hipStream_t s) {
    const int B = p.B, n = p.n;
    // Weight gradients on a side stream s2, each forked after its dOut is final on s.
    // Disjoint from what s writes meanwhile: a dense layer's dOut is its growth slice
    // [coff, coff + g) of dcat, and the BN backward of it and of every earlier layer
    // writes dcat[0, cin) with cin <= coff; the input x is cat (not written in the
    // backward); the slabs and the gradient slots are s2's alone.  The transition dOut
    // buffer dt is shared by the transitions, so s waits for s2 before each pool
    // backward refills it; s waits for everything at the end (Adam reads the gradients).
    hipStream_t s2 = p.side.get(s);
    p.side2.slot = 1;
    hipStream_t s3 = s2 && p.wg2 ? p.side2.get(s) : nullptr;
    p.side3.slot = 2;
    hipStream_t s4 = s3 && p.wgs >= 3 ? p.side3.get(s) : nullptr;
    int wgi = 0;   // weight gradients issued, dealt round-robin over s2, s3 (, s4)
    for (int i = (int)p.layers.size() - 1; i >= 0; --i) {
        Layer& ly = p.layers[i];
        const int st = ly.stage;
        if (ly.kind == K_HEAD) {
            BnArgs bn = bn_args(p, ly, true);
            HeadArgs h = head_args(p, nullptr, nullptr, 0, 0, true);
            bn.bcast = 1; bn.dg = h.dg; bn.dg_ms = h.h_ms; bn.inv_hw = 1.f / (ly.H * ly.W);
            bn.dx = p.act + p.dcat_off[st]; bn.dx_ms = p.cat_ms[st]; bn.dx_ps = p.sC[st]; bn.accumulate = 0;
            enqueue_bn_bwd(p, bn, i, s);
            continue;
        }
        // dOut of this layer's conv and the input it saw
        WgArgs w{};
        w.H = ly.H; w.W = ly.W; w.Cin = ly.cin; w.N = ly.cout; w.R = ly.Rw; w.spg = ly.spg; w.B = B; w.kw = ly.kw;
        const int nws = s4 ? 3 : (s3 ? 2 : 1), ws_i = wgi % nws;
        ++wgi;
        const bool on3 = ws_i == 1, on4 = ws_i == 2;
        w.part = p.act + (on4 ? p.part3_off : on3 ? p.part2_off : p.part_off);
        w.part_ms = on4 ? p.part3_ms : on3 ? p.part2_ms : p.part_ms;
        const float* dout;
        long long dout_ms;
        int dout_ps;
        if (ly.kind == K_TRANS) {
            if (s2) MPO_HIP(p.side.join(s, s2));     // an earlier-issued transition wgrad may still read dt
            if (s3) MPO_HIP(p.side2.join(s, s3));
            if (s4) MPO_HIP(p.side3.join(s, s4));
            const bool v4 = pool_vec4(ly.cout, p.sC[st + 1], p.dt_ms, p.cat_ms[st + 1], p.act + p.dt_off,
                                      p.act + p.dcat_off[st + 1]);
            hipLaunchKernelGGL(v4 ? dn_pool_bwd_kernel<4> : dn_pool_bwd_kernel<1>, dim3((B * ly.H + 1) / 2, n),
                               dim3(256), 0, s, p.act + p.dcat_off[st + 1],
                               p.cat_ms[st + 1], p.sC[st + 1], p.act + p.dt_off, p.dt_ms, B, ly.H, ly.W, ly.cout);
            dout = p.act + p.dt_off; dout_ms = p.dt_ms; dout_ps = ly.cout;
        } else {
            dout = p.act + p.dcat_off[st] + ly.coff; dout_ms = p.cat_ms[st]; dout_ps = p.sC[st];
        }
        w.dout = dout; w.dout_ms = dout_ms; w.dout_ps = dout_ps;
        if (ly.kind == K_CONV0) {
            w.in = x; w.in_ps = ly.cin; w.order = order; w.ord_ms = ord_ms; w.row0 = row0;
            w.img_floats = (long long)ly.H * ly.W * ly.cin;
        } else {
            const BnArgs bx = bn_args(p, ly, true);
            w.in = bx.x; w.in_ms = bx.x_ms; w.in_ps = bx.x_ps;   // cat: the staging forms ELU(BN(x))
            w.bnc = bx.coef; w.bnc_ms = bx.coef_ms;
        }
        hipStream_t sw = s;
        if (on4) {
            MPO_HIP(p.side3.fork(s, s4));
            sw = s4;
        } else if (on3) {
            MPO_HIP(p.side2.fork(s, s3));
            sw = s3;
        } else if (s2) {
            MPO_HIP(p.side.fork(s, s2));
            sw = s2;
        }
        DN_TRY(launch_wgrad(w, ly.ks, n, ly.G, sw));
        const long long cnt = (long long)ly.ks * ly.ks * ly.cin * ly.cout;
        hipLaunchKernelGGL(dn_wgrad_reduce_kernel, flat_grid(cnt, n), dim3(256), 0, sw, (const float*)w.part,
                           w.part_ms, ly.G, cnt, p.grads, p.n_params, ly.w_off);
        if (ly.kind == K_CONV0) continue;
        // input gradient: 'same' conv of dOut with the rotated, transposed kernel -> dz
        BnArgs bn = bn_args(p, ly, true);
        ConvArgs c{};
        c.in = dout; c.in_ms = dout_ms; c.in_ps = dout_ps;
        c.w = p.act + ly.wd_off_act; c.w_ms = ((long long)ly.wd_rows * ly.wd_n16 + 63) & ~63LL;
        c.out = p.act + p.dz_off; c.out_ms = p.dz_ms; c.out_ps = ly.cin;
        c.H = ly.H; c.W = ly.W; c.Cin = ly.cout; c.N = ly.cin; c.R = ly.R;
        c.c1x1 = p.conv1x1 ? 1 : 0;
        const int fS = p.bn_fS[i];
        if (fS > 0) {
            c.rx = bn.x; c.rx_ms = bn.x_ms; c.rx_ps = bn.x_ps;
            c.rcoef = bn.coef; c.rcoef_ms = bn.coef_ms;
            c.rpart = reinterpret_cast<double*>(p.act + p.bnp_off); c.rS = fS;
        }
        if (ly.ks == 3) DN_TRY(launch_conv<3>(c, n, B, s));
        else DN_TRY(launch_conv<1>(c, n, B, s));
        bn.dz = p.act + p.dz_off; bn.dz_ms = p.dz_ms;
        bn.dx = p.act + p.dcat_off[st]; bn.dx_ms = p.cat_ms[st]; bn.dx_ps = p.sC[st];
        bn.accumulate = ly.kind == K_DENSE ? 1 : 0;
        enqueue_bn_bwd(p, bn, i, s, fS);
    }
    if (s2) MPO_HIP(p.side.join(s, s2));
    if (s3) MPO_HIP(p.side2.join(s, s3));
    if (s4) MPO_HIP(p.side3.join(s, s4));
    MPO_LAUNCH_CHECK();
    return MPO_OK;
}

}  // namespace

extern "C" {

int mpo_dn_create(const MpoDnArch* arch, int n_members, int batch, void** handle) {
    MPO_GUARD_BEGIN
    MPO_CHECK_ARG(arch && handle, "mpo_dn_create: null pointer");
    MPO_CHECK_ARG(n_members > 0 && n_members <= 65535 && batch > 0 && batch <= 65535,
                  "mpo_dn_create: n_members %d / batch %d out of range", n_members, batch);
    MPO_CHECK_ARG(arch->depth >= 4 && (arch->depth - 4) % 3 == 0, "mpo_dn_create: Depth must be 3 N + 4 (got %d)",
                  arch->depth);
    MPO_CHECK_ARG(arch->nb_dense_block >= 1 && arch->growth > 0 && arch->nb_filter > 0 && arch->classes > 1 &&
                      arch->H > 0 && arch->W > 0 && arch->C > 0,
                  "mpo_dn_create: bad architecture");
    auto p = std::make_unique<DnPlan>();
    p->arch = *arch;
    p->n = n_members;
    p->B = batch;
    // A/B switch (one variable, as MPO_POP_PLAN for the MNIST population): streams=1
    if (const char* e = getenv("MPO_DN_PLAN")) {
        p->side.enabled = strstr(e, "streams=1") == nullptr;
        p->conv1x1 = strstr(e, "c1x1=0") == nullptr;
        p->wg2 = strstr(e, "wg2=0") == nullptr;
        p->bnfuse = strstr(e, "bnfuse=0") == nullptr;
        if (strstr(e, "wgs=3")) p->wgs = 3;
    }
    const int rc = build_plan(*p);
    if (rc != MPO_OK) {
        mpo::set_error("mpo_dn_create: architecture outside the kernels' range (W <= %d, C <= 1024)", kMaxPix);
        return rc;
    }
    for (auto& ly : p->layers) {
        if (ly.kind == K_HEAD) continue;
        if (conv_lds(ly.R, ly.W, ly.ks, ly.cin) > ((size_t)160 << 10) ||
            conv_lds(ly.R, ly.W, ly.ks, ly.cout) > ((size_t)160 << 10) ||
            wg_lds(ly.Rw, ly.W, ly.ks, ly.cin, (ly.cout + 15) / 16, ly.kw) > ((size_t)160 << 10) || ly.cout > 64 ||
            (ly.kind != K_CONV0 && ly.cin > 96) || (ly.ks == 1 && ly.cin > 64)) {
            mpo::set_error("mpo_dn_create: layer (cin %d, cout %d, %dx%d) exceeds the kernels' LDS / channel range",
                           ly.cin, ly.cout, ly.H, ly.W);
            return MPO_ENOTSUP;
        }
    }
    *handle = p.release();
    return MPO_OK;
    MPO_GUARD_END
}

int mpo_dn_destroy(void* handle) {
    delete static_cast<DnPlan*>(handle);
    return MPO_OK;
}

int mpo_dn_sizes(const void* handle, MpoDnSizes* out) {
    MPO_CHECK_ARG(handle && out, "mpo_dn_sizes: null pointer");
    const DnPlan& p = *static_cast<const DnPlan*>(handle);
    out->n_params = p.n_params;
    out->n_state = p.n_state;
    out->act_floats = p.act_floats;
    out->n_members = p.n;
    out->batch = p.B;
    out->n_layers = (int32_t)p.layers.size();
    return MPO_OK;
}

int mpo_dn_layer(const void* handle, int i, int32_t* geom, int64_t* offs) {
    MPO_CHECK_ARG(handle && geom && offs, "mpo_dn_layer: null pointer");
    const DnPlan& p = *static_cast<const DnPlan*>(handle);
    MPO_CHECK_ARG(i >= 0 && i < (int)p.layers.size(), "mpo_dn_layer: layer %d out of range", i);
    const Layer& ly = p.layers[i];
    const int32_t g[8] = {ly.kind, ly.stage, ly.H, ly.W, ly.cin, ly.cout, ly.ks, ly.coff};
    for (int k = 0; k < 8; ++k) geom[k] = g[k];
    const bool head = ly.kind == K_HEAD;
    const int64_t o[6] = {head ? p.wd_off : ly.w_off, ly.g_off, ly.b_off, ly.mm_off, ly.mv_off, head ? p.bd_off : -1};
    for (int k = 0; k < 6; ++k) offs[k] = o[k];
    return MPO_OK;
}

int mpo_dn_bind(void* handle, float* params, float* grads, float* adam_m, float* adam_v, float* state, float* act,
                const float* lr, void* stream) {
    MPO_GUARD_BEGIN
    MPO_CHECK_ARG(handle && params && grads && adam_m && adam_v && state && act && lr, "mpo_dn_bind: null pointer");
    DnPlan& p = *static_cast<DnPlan*>(handle);
    p.params = params; p.grads = grads; p.m = adam_m; p.v = adam_v; p.state = state; p.act = act;
    MPO_HIP(hipMemcpyAsync(act + p.lr_off, lr, sizeof(float) * p.n, hipMemcpyHostToDevice,
                           static_cast<hipStream_t>(stream)));
    MPO_HIP(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
    p.bound = true;
    return MPO_OK;
    MPO_GUARD_END
}

int mpo_dn_train_step(void* handle, const float* x, const int32_t* labels, const int32_t* order, int64_t order_stride,
                      int64_t row0, int32_t step, float* loss_out, void* stream) {
    MPO_GUARD_BEGIN
    MPO_CHECK_ARG(handle && x && labels && order && loss_out, "mpo_dn_train_step: null pointer");
    DnPlan& p = *static_cast<DnPlan*>(handle);
    MPO_CHECK_ARG(p.bound, "mpo_dn_train_step: plan not bound");
    MPO_CHECK_ARG(step >= 0 && row0 >= 0 && row0 + p.B <= order_stride, "mpo_dn_train_step: batch outside the order table");
    hipStream_t s = static_cast<hipStream_t>(stream);
    DN_TRY(enqueue_prep(p, true, s));
    DN_TRY(enqueue_forward(p, x, labels, order, order_stride, row0, true, loss_out, nullptr, nullptr, s));
    DN_TRY(enqueue_backward(p, x, order, order_stride, row0, s));
    hipLaunchKernelGGL(dn_adam_kernel, flat_grid(p.n_params, p.n), dim3(256), 0, s, p.params, p.grads, p.m, p.v,
                       p.n_params, p.n_params, (const float*)(p.act + p.lr_off), (int)step + 1);
    MPO_LAUNCH_CHECK();
    return MPO_OK;
    MPO_GUARD_END
}

int mpo_dn_eval_step(void* handle, const float* x, const int32_t* labels, const int32_t* order, int64_t order_stride,
                     int64_t row0, float* loss_sum, int32_t* correct, void* stream) {
    MPO_GUARD_BEGIN
    MPO_CHECK_ARG(handle && x && labels && order && loss_sum && correct, "mpo_dn_eval_step: null pointer");
    DnPlan& p = *static_cast<DnPlan*>(handle);
    MPO_CHECK_ARG(p.bound, "mpo_dn_eval_step: plan not bound");
    MPO_CHECK_ARG(row0 >= 0 && row0 + p.B <= order_stride, "mpo_dn_eval_step: batch outside the order table");
    hipStream_t s = static_cast<hipStream_t>(stream);
    DN_TRY(enqueue_prep(p, false, s));
    DN_TRY(enqueue_forward(p, x, labels, order, order_stride, row0, false, nullptr, loss_sum, correct, s));
    return MPO_OK;
    MPO_GUARD_END
}

int mpo_dn_penalty(void* handle, float* out, void* stream) {
    MPO_GUARD_BEGIN
    MPO_CHECK_ARG(handle && out, "mpo_dn_penalty: null pointer");
    DnPlan& p = *static_cast<DnPlan*>(handle);
    MPO_CHECK_ARG(p.bound, "mpo_dn_penalty: plan not bound");
    hipLaunchKernelGGL(dn_penalty_kernel, dim3(p.n), dim3(256), 0, static_cast<hipStream_t>(stream), p.params,
                       p.n_params, p.n_params, out);
    MPO_LAUNCH_CHECK();
    return MPO_OK;
    MPO_GUARD_END
}

}  // extern "C"
