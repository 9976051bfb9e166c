// cnn.hip -- population training of ragged MNIST-CNN trials on gfx950 (MI355X).
//
// Hot path T2-T6 of SURVEY §8a: replaces ProcessBlock.train_model ->
// mpi_learn MPIKFoldManager (/root/reference/process_block.py:71-96) for the
// test_mnist model (/root/reference/mpiLAPI.py:138-176).  Every member of the
// population is one (trial, fold) pair with its own widths (F, k, p, dense),
// learning rate, dropout rate and dropout seed; one launch per op covers every
// member through a host-built work list (grouped / ragged launches).
//
// Per training step (all members, batch B):
//   conv_img<CONV1_FWD>   x[order] (k-fold index gather) -> a1 = relu(conv1)
//   conv_img<CONV2_FWD>   a1 -> a2 = relu(conv2)
//   pool_fwd              a2 -> pd = dropout(maxpool(a2)), argmax
//   dense<D1_FWD>         pd -> h = relu(pd w3 + b3), hd = dropout(h)
//   dense<D2_FWD>         hd -> z3 = hd w4 + b4
//   softmax_bce           z3 -> loss, dz3
//   dense<D2_WGRAD/DGRAD> dw4;  dh = dz3 w4^T * mask * (h>0)
//   dense<D1_WGRAD/DGRAD> dw3;  dp = dh w3^T * mask
//   pool_bwd              dp -> dz2 = unpool(dp) * (a2>0)
//   flip_w2               w2 -> w2t (rotated, in/out swapped: dgrad weights)
//   conv_img<CONV2_DGRAD> dz2 (virtually zero-padded) -> dz1 = conv(dz2, w2t) * (a1>0)
//   conv_wgrad<CONV2>     a1, dz2 -> dw2 partial slabs (per sample group)
//   conv_wgrad<CONV1>     x[order], dz1 -> dw1 partial slabs
//   wgrad_reduce, colsum  slabs -> dw1, dw2; bias grads
//   adam                  per-member lr, Keras-form Adam
//
// The convolutions are image-stationary implicit GEMMs: a workgroup stages
// the input rows it needs for one sample (and one output row chunk) into LDS
// once, and every MFMA A-fragment is an LDS gather at (pixel base + tap
// offset) -- no im2col buffer, no k^2 re-reads from L2.  Arithmetic is f32 on
// v_mfma_f32_16x16x4_f32 (exact f32, the reference's precision).

#include "mpo_internal.h"

#include <algorithm>
#include <cstring>
#include <cmath>
#include <cstdlib>
#include <memory>
#include <string>
#include <type_traits>
#include <vector>

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kImg = 28;
constexpr int kClasses = 10;
constexpr float kBceEps = 1e-7f;

// ---- device member descriptor (mirrors the host plan) ----------------------
struct Member {
    int F, k, p, dense;
    int H1, H2, s, K1;
    float lr, rate, inv_keep;
    int loss, opt;      // MPO_LOSS_*, MPO_OPT_* (MpoCnnSpec.options)
    unsigned seed;
    unsigned drop_thr;  // keep iff (hash >> 8) >= drop_thr
    int nt;             // ceil(F / 16)
    int g1, g2;         // wgrad sample groups (conv1, conv2)
    // parameter arena offsets (floats); the same offsets index grads / adam m / v
    long long w1, b1, w2, b2, w3, b3, w4, b4, pend;
    // activation arena offsets (floats)
    long long a1, a2, pd, am, h, hd, z3, dz3, dh, dp, dz2, dz1, w2t, wp1, wp2;
    long long w1p, w2p;  // zero-padded forward weights [K16 + kWSlack][16*NT]
};

struct ConvItem { int member, b, y0, R; };
struct WgItem { int member, mg, b0, b1, group, R; };
struct GemmItem { int member, m0, n0, pad; };
struct MItem { int member, aux; };

enum ConvOp { CONV1_FWD = 0, CONV2_FWD = 1, CONV2_DGRAD = 2 };
enum WgOp { WG_CONV1 = 0, WG_CONV2 = 1 };
enum DenseOp { D1_FWD = 0, D2_FWD = 1, D2_WGRAD = 2, D2_DGRAD = 3, D1_WGRAD = 4, D1_DGRAD = 5 };

struct StepArgs {
    const Member* mem;
    const float* params;
    float* grads;
    float* act;
    const float* x;          // [n_samples][784]
    const int* labels;       // [n_samples]
    const int* order;        // sample order per member
    long long order_stride;  // entries per member row
    long long row0;          // first row of this batch in the order
    int B;
    int step;                // dropout stream position
    int train;               // 1 = training (dropout on), 0 = eval
    float* loss_out;         // [n_members] mean batch loss (train)
    float* loss_sum;         // [n_members] running loss sum (eval)
    int* correct;            // [n_members] running correct count (eval)
    long long zero_off;      // 64 zero floats in the activation arena (DMA source past row ends)
    int debug;               // diagnostics only (env MPO_POP_DEBUG / plan dbg): 1 skip conv MMA loops, 2 skip conv staging,
                             // 4 conv fwd / dgrad weight fragments re-read from groups 0-1 (cache-resident; timing only)
    int conv_mt;             // forward conv m-tiles per wave at most (2: M <= 128 pixels per item; 4: <= 256)
    int wgrpb;               // conv2 weight gradient: output rows per barrier (1 | 2)
    int wgpair;              // wgrpb 2 and Ho = 2 (mod 4): a row pair as one K run (plan knob wgpair)
};


// ---- dropout counter hash (identical in oracle/cnn.py) ---------------------
__device__ __forceinline__ unsigned lowbias32(unsigned x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

__device__ __forceinline__ unsigned drop_base(unsigned seed, int step, int layer) {
    unsigned b = lowbias32(seed ^ (unsigned)(layer * 0x9E3779B9u));
    return lowbias32(b ^ (unsigned)step);
}

__device__ __forceinline__ bool drop_keep(unsigned base, unsigned elem, unsigned thr) {
    return (lowbias32(elem ^ base) >> 8) >= thr;
}

// LDS pixel strides chosen for conflict-free MFMA operand reads (ds_read_b32 banks
// = dword index mod 32 per 32-lane half):
//  * forward conv: lanes 0-15 read 16 pixels at stride fp, lanes 16-31 the next
//    channel (+1): fp = 2 (mod 4) puts the two halves on the even / odd banks;
__host__ __device__ constexpr inline int fwd_fp(int c) { return c == 1 ? 1 : c + ((6 - (c & 3)) & 3); }
//  * and the LDS row stride = Ho * fp (mod 32): output pixel m = y*Ho + x then sits at
//    m * fp (mod 32), so a 16-pixel tile that wraps to the next row stays on 16
//    distinct banks (a Wp * fp stride shifts the wrapped part by (k-1) * fp).
//    conv1 (one channel, taps on adjacent lanes) keeps the plain Wp stride.
__host__ __device__ constexpr inline int fwd_rs(int Wp, int Cin, int Ho) {
    return Cin == 1 ? Wp : Wp * fwd_fp(Cin) + ((Ho * fwd_fp(Cin) - Wp * fwd_fp(Cin)) & 31);
}

// ============================================================================
// Image-stationary implicit-GEMM convolution (forward and input-gradient).
//   out[b][y][x][n] = sum_{ky,kx,c} in_pad[b][y+ky][x+kx][c] * W[(ky*k+kx)*Cin+c][n]
// One workgroup = (member, sample b, output rows [y0, y0+R)); M = R*Ho <= 64*MTX
// output pixels = 4*MTX m-tiles of 16 spread over 4 waves; N = F in NT tiles of 16.
// ============================================================================

__host__ __device__ constexpr inline int align4(int x) { return (x + 3) & ~3; }

// dgrad image pixel stride: >= F rounded to 4 (zero channels for the 16-channel
// k blocks) and = 2 (mod 4), which makes the 4x4-tile A reads bank-conflict free.
__host__ __device__ constexpr inline int dgrad_fp(int F) { return ((F + 3) & ~3) + 2; }

// dgrad LDS row stride: >= H2 * Fp and = 8 (mod 32).  A 4x4 patch reads rows dy at
// dy * RS and columns dx at dx * Fp: with Fp = 2 (mod 4) the columns take the four
// even residues mod 8 and the rows the four multiples of 8, so the 16 pixels (and
// the next channel, +1, on the odd banks) are conflict-free.  An unpadded H2 * Fp is
// = 0 or 16 (mod 32) (H2 even) and put rows dy and dy + 2 on the same banks.
__host__ __device__ constexpr inline int dgrad_rs(int H2, int F) {
    return H2 * dgrad_fp(F) + ((8 - ((H2 * dgrad_fp(F)) & 31)) & 31);
}

// Copy rows x w pixels x cin channels of contiguous floats (NHWC rows of one
// sample) into an LDS image with pixel stride fp and row stride rs.  The element
// walk (row, pixel, channel) advances by mixed-radix adds (no per-element integer
// division), and every thread issues kStageBatch loads before their LDS stores:
// r03 -- a load-then-store loop per row kept ONE global load per thread in flight,
// and the staging ran ~13 us per conv work item.
constexpr int kStageBatch = 8;
__device__ __forceinline__ void stage_rows(const float* __restrict__ src, float* __restrict__ dst, int rows, int w,
                                           int cin, int fp, int rs, int tid) {
    const int n = rows * w * cin;
    int c = tid % cin, t = tid / cin;
    int x = t % w, r = t / w;
    const int sc = 256 % cin, st = 256 / cin, sx = st % w, sr = st / w;
    auto adv = [&]() {
        c += sc;
        int cx = 0;
        if (c >= cin) { c -= cin; cx = 1; }
        x += sx + cx;
        int cr = 0;
        if (x >= w) { x -= w; cr = 1; }
        r += sr + cr;
    };
    int e = tid;
    for (; e + (kStageBatch - 1) * 256 < n; e += kStageBatch * 256) {
        float v[kStageBatch];
        int d[kStageBatch];
#pragma unroll
        for (int u = 0; u < kStageBatch; ++u) v[u] = src[e + u * 256];
#pragma unroll
        for (int u = 0; u < kStageBatch; ++u) {
            d[u] = r * rs + x * fp + c;
            adv();
        }
#pragma unroll
        for (int u = 0; u < kStageBatch; ++u) dst[d[u]] = v[u];
    }
    for (; e < n; e += 256) {
        dst[r * rs + x * fp + c] = src[e];
        adv();
    }
}

// Slack past the K16 rows: the pipelined loops below run an even number of
// 16-k groups and read up to two groups (weights) and three groups (tap
// offsets) past that; the slack is zero.
constexpr int kWSlack = 48;
constexpr int kKoffSlack = 64;

// Main loop of the forward conv for MT (<= MTX) m-tiles per wave: one 16-k group
// per half-iteration; the weights of group g+1 (L2 -> VGPR) and the A gathers of
// group g+1 (LDS) are issued before the MFMAs of group g, and the tap offsets
// one group further ahead, so no MFMA waits on a load issued in its own group.
template <int MT, int NT, int MTX>
__device__ __forceinline__ void conv_fwd_loop(const float* __restrict__ img, const int* __restrict__ koff,
                                              const float* __restrict__ W, int ngroups, const int (&pb)[MTX],
                                              f32x4 (&acc)[MTX][NT], int krow, int kcol, int gmask) {
    constexpr int N16 = NT * 16;
    const float* wsrc = W + krow * N16 + kcol;
    const int* kp = koff + krow * 4;
    float b0[4][NT], b1[4][NT], a0[4][MT], a1[4][MT];
    auto loadB = [&](int g, float (&dst)[4][NT]) {
        const float* src = wsrc + (long long)(g & gmask) * 16 * N16;
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
    loadB(0, b0);
    int4 ko = kof(0);
    readA(ko, a0);
    ko = kof(1);
    // Two groups per iteration with no exit in between (an odd group count runs
    // one zero group from the slack): a mid-loop exit makes the compiler shuffle
    // the accumulators between AGPRs at every iteration.  sched_barrier(0) pins
    // the issue order -- otherwise each load sinks next to its first use.
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

template <int OP, int NT, int MTX>
__global__ __launch_bounds__(256) void conv_img_kernel(StepArgs a, const ConvItem* __restrict__ items) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const ConvItem it = items[blockIdx.x];
    const Member& mb = a.mem[it.member];
    const int k = mb.k, F = mb.F;
    int Hin, Cin, Ho;
    const float* in;
    const float* W;
    const float* bias = nullptr;
    float* out;
    const float* relu_mask = nullptr;
    if (OP == CONV2_DGRAD) {
        // r06: the conv2 input gradient as a forward conv over dz2 zero-bordered by k - 1
        // (Hin = H2 + 2 (k - 1) = H1 + k - 1), the rotated weights w2t, Cin = F rounded to
        // 4 (w2t's channel stride; channels >= F are zero in the image and in w2t).  Every
        // MFMA step multiplies the same 4 (tap, channel) pairs as conv_dgrad_kernel's;
        // the halo steps it does not skip only add exact zeros: the same bits.
        Hin = mb.H1 + k - 1; Cin = (F + 3) & ~3; Ho = mb.H1;
        in = a.act + mb.dz2 + (long long)it.b * mb.H2 * mb.H2 * F;
        W = a.act + mb.w2t;
        out = a.act + mb.dz1 + (long long)it.b * Ho * Ho * F;
        relu_mask = a.act + mb.a1 + (long long)it.b * Ho * Ho * F;
    } else if (OP == CONV1_FWD) {
        Hin = kImg; Cin = 1; Ho = mb.H1;
        const int sidx = a.order[(long long)it.member * a.order_stride + a.row0 + it.b];
        in = a.x + (long long)sidx * (kImg * kImg);
        W = a.act + mb.w1p; bias = a.params + mb.b1;
        out = a.act + mb.a1 + (long long)it.b * Ho * Ho * F;
    } else {
        Hin = mb.H1; Cin = F; Ho = mb.H2;
        in = a.act + mb.a1 + (long long)it.b * Hin * Hin * F;
        W = a.act + mb.w2p; bias = a.params + mb.b2;
        out = a.act + mb.a2 + (long long)it.b * Ho * Ho * F;
    }
    const int N = F;
    const int K = k * k * Cin;
    const int K16 = (K + 15) & ~15;
    const int Wp = Hin;
    const int Fp = fwd_fp(Cin);
    const int rows = it.R + k - 1;
    const int M = it.R * Ho;

    float* img = smem;                                               // [rows][Wp][Fp]
    const int RS = fwd_rs(Wp, Cin, Ho);
    const int img_elems = rows * RS;
    int* koff = reinterpret_cast<int*>(smem + align4(img_elems));   // [K16 + slack], groups of 16 as [krow][4]
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int krow = lane >> 4, kcol = lane & 15;

    // ---- stage the input rows + the tap-offset table (the only barrier)
    if (OP == CONV2_DGRAD) {
        // zero image (halo rows / columns, channels >= F), then dz2's rows inside it:
        // padded row y0 + r is dz2 row y0 + r - (k - 1)
        const int pad = k - 1, H2 = mb.H2;
        for (int e = tid; e < img_elems; e += 256) img[e] = 0.f;
        __syncthreads();
        const int gy_lo = max(0, it.y0 - pad), gy_hi = min(H2, it.y0 + it.R);
        if (a.debug != 2 && gy_hi > gy_lo)
            stage_rows(in + (long long)gy_lo * H2 * F, img + (gy_lo + pad - it.y0) * RS + pad * Fp, gy_hi - gy_lo, H2,
                       F, Fp, RS, tid);
    } else if (a.debug != 2) {
        const float* src = in + (long long)it.y0 * Hin * Cin;
        if (Cin == 1) {
            for (int e = tid; e < rows * Hin; e += 256) {
                const int r = e / Hin;
                img[r * RS + e - r * Hin] = src[e];
            }
        } else {
            stage_rows(src, img, rows, Hin, Cin, Fp, RS, tid);
        }
    }
    for (int kk = tid; kk < K16 + kKoffSlack; kk += 256) {
        int off = 0;
        if (kk < K) {
            const int kc = k * Cin;
            const int ky = kk / kc, rem = kk - ky * kc;
            const int kx = rem / Cin, c = rem - kx * Cin;
            off = ky * RS + kx * Fp + c;
        }
        const int g = kk >> 4, w = kk & 15;        // k = 16 g + 4 u + krow
        koff[g * 16 + (w & 3) * 4 + (w >> 2)] = off;
    }

    const int mtiles = (M + 15) >> 4;
    // m-tile t is wave t % 4's slot t / 4
    const int mine = __builtin_amdgcn_readfirstlane(mtiles > wave ? min(MTX, (mtiles - wave + 3) >> 2) : 0);
    int pb[MTX];
#pragma unroll
    for (int i = 0; i < MTX; ++i) {
        const int m = (wave + 4 * i) * 16 + (lane & 15);
        int base = 0;
        if (m < M) {
            const int y = m / Ho, xx = m - y * Ho;
            base = y * RS + xx * Fp;
        }
        pb[i] = base;
    }
    f32x4 acc[MTX][NT];
#pragma unroll
    for (int i = 0; i < MTX; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    __syncthreads();
    const int ngroups = a.debug == 1 ? 0 : K16 >> 4;
    const int gmask = a.debug == 4 ? 1 : -1;
    if constexpr (MTX == 4) {
        if (mine == 4) conv_fwd_loop<4, NT, MTX>(img, koff, W, ngroups, pb, acc, krow, kcol, gmask);
        else if (mine == 3) conv_fwd_loop<3, NT, MTX>(img, koff, W, ngroups, pb, acc, krow, kcol, gmask);
        else if (mine == 2) conv_fwd_loop<2, NT, MTX>(img, koff, W, ngroups, pb, acc, krow, kcol, gmask);
        else if (mine == 1) conv_fwd_loop<1, NT, MTX>(img, koff, W, ngroups, pb, acc, krow, kcol, gmask);
        else return;
    } else {
        if (mine == 2) conv_fwd_loop<2, NT, MTX>(img, koff, W, ngroups, pb, acc, krow, kcol, gmask);
        else if (mine == 1) conv_fwd_loop<1, NT, MTX>(img, koff, W, ngroups, pb, acc, krow, kcol, gmask);
        else return;
    }

    // ---- epilogue: C/D map col = lane & 15, row = (lane >> 4) * 4 + r
    const long long pix0 = (long long)it.y0 * Ho;
#pragma unroll
    for (int i = 0; i < MTX; ++i) {
        if (i >= mine) break;
        const int mt = wave + 4 * i;
#pragma unroll
        for (int j = 0; j < NT; ++j) {
            const int n = j * 16 + kcol;
            if (n >= N) continue;
            const float bv = OP == CONV2_DGRAD ? 0.f : bias[n];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = mt * 16 + krow * 4 + r;
                if (m >= M) continue;
                const long long o = (pix0 + m) * N + n;
                if (OP == CONV2_DGRAD) out[o] = relu_mask[o] > 0.f ? acc[i][j][r] : 0.f;
                else out[o] = fmaxf(acc[i][j][r] + bv, 0.f);
            }
        }
    }
}

// ============================================================================
// Input gradient of conv2 (tap-major, halo-skipping):
//   dz1[b][y][x][c] = (a1 > 0) * sum_{ky',kx',f} dz2pad[y+ky'][x+kx'][f] * w2t[(ky',kx',f)][c]
// dz2pad is dz2 with a virtual zero halo of k-1; w2t the rotated weights.  Each
// 16-pixel MFMA tile is a 4x4 spatial patch, so a tap whose receptive field lies
// entirely in the halo for that patch is skipped (wave-uniform branch) -- the
// padded formulation otherwise multiplies zeros for (H1/H2)^2 of its work.
// The halo is virtual in the LDS too: only the dz2 rows the chunk reads are
// staged (unpadded, [rows][H2][Fp]); a lane whose tap pixel falls in the halo
// reads a zero block instead.  (A padded image is up to 5x larger at k=10 and
// capped the chunk at 4 rows -- 5 tiles on 4 waves.)
// One workgroup = (member, sample, output rows [y0, y0+R)), R = 4*floor(16/CT)
// (<= 16 tiles of 4x4, at most 4 per wave); K loop = (tap, 16-channel block).
// ============================================================================
template <int NT>
__global__ __launch_bounds__(256) void conv_dgrad_kernel(StepArgs a, const ConvItem* __restrict__ items) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const ConvItem it = items[blockIdx.x];
    const Member& mb = a.mem[it.member];
    const int k = mb.k, F = mb.F, H2 = mb.H2, Ho = mb.H1;
    const int pad = k - 1;
    const int F4 = (F + 3) & ~3;
    const int Fp = dgrad_fp(F);
    const int N = F;
    const int R = it.R, y0 = it.y0;
    const int gy_lo = max(0, y0 - pad), gy_hi = min(H2, y0 + R);   // dz2 rows read by this chunk
    const int rows = gy_hi - gy_lo;
    const float* in = a.act + mb.dz2 + (long long)it.b * H2 * H2 * F;
    const float* W = a.act + mb.w2t;
    float* out = a.act + mb.dz1 + (long long)it.b * Ho * Ho * F;
    const float* relu_mask = a.act + mb.a1 + (long long)it.b * Ho * Ho * F;

    float* img = smem;  // [rows][RS] (H2 pixels of Fp), channels >= F zero; then a 64-float zero block
    const int RS = dgrad_rs(H2, F);
    const int zoff = align4(rows * RS);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: tile logic stays scalar
    const int krow = lane >> 4, kcol = lane & 15;

    for (int e = tid; e < zoff + 64; e += 256) img[e] = 0.f;
    __syncthreads();
    if (a.debug != 2) stage_rows(in + (long long)gy_lo * H2 * F, img, rows, H2, F, Fp, RS, tid);

    // ---- this wave's 4x4 tiles, their tap rectangles and the wave's union rectangle
    const int CT = (Ho + 3) >> 2;
    const int bands = (R + 3) >> 2;
    const int T = bands * CT;
    // contiguous tiles per wave (neighbours along a band share most live taps, so the
    // wave's union tap rectangle wastes fewer groups than a round-robin spread)
    const int per = (T + 3) >> 2;
    int py[4], px[4], kylo[4], kyhi[4], kxlo[4], kxhi[4];
    bool has[4];
    int uy0 = k, uy1 = 0, ux0 = k, ux1 = 0;
    const int dy = (lane & 15) >> 2, dx = lane & 3;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int ti = wave * per + i;
        has[i] = i < per && ti < T;
        const int band = ti / CT, ct = ti - band * CT;
        const int ty0 = y0 + 4 * band, tx0 = 4 * ct;
        const int ty1 = min(ty0 + 4, y0 + R), tx1 = min(tx0 + 4, Ho);
        kylo[i] = max(0, pad - (ty1 - 1));
        kyhi[i] = min(k, pad + H2 - ty0);
        kxlo[i] = max(0, pad - (tx1 - 1));
        kxhi[i] = min(k, pad + H2 - tx0);
        if (has[i]) {
            uy0 = min(uy0, kylo[i]); uy1 = max(uy1, kyhi[i]);
            ux0 = min(ux0, kxlo[i]); ux1 = max(ux1, kxhi[i]);
        }
        // tap (ky, kx) reads dz2 pixel (y + ky - pad, x + kx - pad): LDS row py + ky, column px + kx
        const int y = ty0 + dy, x = tx0 + dx;
        const bool pix = y < ty1 && x < tx1;
        py[i] = pix ? y - pad - gy_lo : -(1 << 20);   // an invalid output pixel never reads the image
        px[i] = x - pad;
    }
    f32x4 acc[4][NT];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    __syncthreads();  // image staged; no further barriers

    // Weight fragments straight from L2: group = (tap, 16-channel block), 4 k-steps;
    // ping-pong register buffers (loop unrolled by two), loads unconditional.
    const int CB = (F4 + 15) >> 4;
    const int nx = ux1 - ux0;
    const int ngroups = (uy1 > uy0 && nx > 0 && a.debug != 1) ? (uy1 - uy0) * nx * CB : 0;
    constexpr int N16 = NT * 16;
    auto load_group = [&](int ky, int kx, int cb, float (&dst)[4][NT]) {
        // w2t is [k*k][F4][N16], zero padded (+16 rows of slack): no bounds select,
        // so the loads stay in flight until the MFMAs of the group consume them
        const float* src = W + ((long long)(a.debug == 4 ? (cb & 1) * 16 : (ky * k + kx) * F4 + cb * 16) + krow) * N16 + kcol;
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int j = 0; j < NT; ++j) dst[u][j] = src[u * 4 * N16 + j * 16];
    };
    auto advance = [&](int& ky, int& kx, int& cb) {
        if (++cb == CB) { cb = 0; if (++kx == ux1) { kx = ux0; ++ky; } }
    };
    // A fragments of a group: 4 k-steps x 4 tiles, read from the LDS image one group
    // ahead of their MFMAs (like the B fragments), so no MFMA waits on its own reads
    auto readA = [&](int ky, int kx, int cb, float (&av)[4][4]) {
        const int coff = cb * 16 + krow;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int ry = py[i] + ky, cx = px[i] + kx;
            const int base = ((unsigned)ry < (unsigned)rows && (unsigned)cx < (unsigned)H2)
                                 ? ry * RS + cx * Fp + coff : zoff + krow;   // halo -> zero block
#pragma unroll
            for (int u = 0; u < 4; ++u) av[u][i] = img[base + u * 4];
        }
    };
    auto compute = [&](int ky, int kx, int cb, const float (&av)[4][4], const float (&bw)[4][NT]) {
        bool live[4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
            live[i] = has[i] && ky >= kylo[i] && ky < kyhi[i] && kx >= kxlo[i] && kx < kxhi[i];
        const int nu = min(4, (F4 - cb * 16) >> 2);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (u >= nu) break;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                if (!live[i]) continue;
#pragma unroll
                for (int j = 0; j < NT; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u][i], bw[u][j], acc[i][j], 0, 0, 0);
            }
        }
    };
    float b0[4][NT], b1[4][NT], a0[4][4], a1[4][4];
    int cky = uy0, ckx = ux0, ccb = 0;   // group g
    int nky = uy0, nkx = ux0, ncb = 0;   // group g + 1
    if (ngroups) {
        load_group(cky, ckx, ccb, b0);
        readA(cky, ckx, ccb, a0);
        advance(nky, nkx, ncb);
    }
    for (int g = 0; g < ngroups; g += 2) {
        if (g + 1 < ngroups) {
            load_group(nky, nkx, ncb, b1);
            readA(nky, nkx, ncb, a1);
        }
        __builtin_amdgcn_sched_barrier(0);
        compute(cky, ckx, ccb, a0, b0);
        __builtin_amdgcn_sched_barrier(0);
        if (g + 1 >= ngroups) break;
        cky = nky; ckx = nkx; ccb = ncb;
        advance(nky, nkx, ncb);
        if (g + 2 < ngroups) {
            load_group(nky, nkx, ncb, b0);
            readA(nky, nkx, ncb, a0);
        }
        __builtin_amdgcn_sched_barrier(0);
        compute(cky, ckx, ccb, a1, b1);
        __builtin_amdgcn_sched_barrier(0);
        cky = nky; ckx = nkx; ccb = ncb;
        advance(nky, nkx, ncb);
    }

    // ---- epilogue: accumulator row p = krow*4 + r is tile pixel (p>>2, p&3)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if (!has[i]) continue;
        const int ti = wave * per + i;
        const int band = ti / CT, ct = ti - band * CT;
        const int ty0 = y0 + 4 * band, tx0 = 4 * ct;
        const int ty1 = min(ty0 + 4, y0 + R), tx1 = min(tx0 + 4, Ho);
#pragma unroll
        for (int j = 0; j < NT; ++j) {
            const int n = j * 16 + kcol;
            if (n >= N) continue;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int p = krow * 4 + r;
                const int y = ty0 + (p >> 2), x = tx0 + (p & 3);
                if (y >= ty1 || x >= tx1) continue;
                const long long o = ((long long)y * Ho + x) * N + n;
                out[o] = relu_mask[o] > 0.f ? acc[i][j][r] : 0.f;
            }
        }
    }
}


// ============================================================================
// Weight gradient: dW[(ky,kx,c)][n] = sum_{b,y,x} in[b][y+ky][x+kx][c] * dout[b][y][x][n]
// (plus the bias gradient as row Kw = k*k*Cin: an all-ones A row).
// GEMM view M = Kw + 1 rows of (ky,kx,c), N = F, K = pixels.  One workgroup =
// (member, 512-row m-group, a group of samples), 8 waves x up to 4 m-tiles.
// The workgroup streams its samples one OUTPUT ROW at a time.  Output row y
// needs input rows y .. y+k-1: they live in an LDS ring of k+2 row slots, each
// input row staged exactly once per m-group; the dout rows in 3 buffers.  Rows
// arrive by LDS-DMA (global_load_lds_dword) two output rows ahead: at row y the
// workgroup issues input row y+k+1 and dout row y+2, waits (counted vmcnt) for
// what it issued at row y-1 and meets one raw s_barrier -- the DMA stays in
// flight across the barrier, so its latency hides behind two rows of MFMAs.
// Every wave issues exactly kWgDma DMA instructions per row (lanes past a row's
// end read a zero block), so the counted wait is a constant.
// Writes one partial slab per sample group (reduced in fixed order later).
// ============================================================================
constexpr int kWgWaves = 8;
constexpr int kWgThreads = kWgWaves * 64;
constexpr int kWgMaxMT = 4;                        // m-tiles per wave
constexpr int kWgRows = kWgWaves * kWgMaxMT * 16;  // 512 rows per m-group
constexpr int kWgChunks = 4;                       // 64-float DMA chunks per wave per row: rows <= 8*4*64 floats
// DMA instructions per wave per output row: 2 * kWgChunks = 8 (the vmcnt(8) below)
static_assert(kWgChunks == 4, "the counted s_waitcnt vmcnt(8) assumes 2 * 4 DMA instructions per row");

typedef __attribute__((address_space(3))) void* lds_ptr_t;

__host__ __device__ constexpr inline int round64(int x) { return (x + 63) & ~63; }

// One output row's MFMAs for MT m-tiles: nk4 k-steps of 4 pixels; the LDS reads
// of k-step s+1 are issued before the MFMAs of k-step s.
template <int MT, int NT>
__device__ __forceinline__ void wgrad_row(const float* __restrict__ img, const float* __restrict__ dl,
                                          const int (&abase)[MT], const int (&astep)[MT], int dstride,
                                          int nk4, int krow, int kcol, f32x4 (&acc)[MT][NT]) {
    float a0[MT], a1[MT], b0[NT], b1[NT];
    auto rd = [&](int s, float (&av)[MT], float (&bv)[NT]) {
        const int x = 4 * s + krow;
#pragma unroll
        for (int i = 0; i < MT; ++i) av[i] = img[abase[i] + x * astep[i]];
#pragma unroll
        for (int j = 0; j < NT; ++j) bv[j] = dl[x * dstride + j * 16 + kcol];
    };
    auto mma = [&](const float (&av)[MT], const float (&bv)[NT]) {
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int j = 0; j < NT; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i], bv[j], acc[i][j], 0, 0, 0);
    };
    rd(0, a0, b0);
    for (int s = 0; s < nk4; s += 2) {
        rd(s + 1, a1, b1);   // s + 1 <= nk4: reads zero dout padding / finite LDS
        __builtin_amdgcn_sched_barrier(0);
        mma(a0, b0);
        __builtin_amdgcn_sched_barrier(0);
        if (s + 1 >= nk4) break;
        rd(s + 2, a0, b0);
        __builtin_amdgcn_sched_barrier(0);
        mma(a1, b1);
        __builtin_amdgcn_sched_barrier(0);
    }
}

// Two output rows as ONE K run of 2 Ho pixels (RPB = 2, Ho = 2 (mod 4)): pixel x of
// the pair is row x >= Ho's pixel x - Ho (a per-lane select), so no k-step straddles
// zero padding -- row-by-row, ceil(Ho / 4) steps per row multiply 2 padding pixels
// (Ho = 10: 6 steps for 10 pixels).  The pair's run: 2 Ho / 4 steps.
template <int MT, int NT>
__device__ __forceinline__ void wgrad_row_pair(const float* __restrict__ img, const float* __restrict__ dl0,
                                               const float* __restrict__ dl1, const int (&abase0)[MT],
                                               const int (&abase1)[MT], const int (&astep)[MT], int dstride, int Ho,
                                               int nk, int krow, int kcol, f32x4 (&acc)[MT][NT]) {
    float a0[MT], a1[MT], b0[NT], b1[NT];
    auto rd = [&](int s, float (&av)[MT], float (&bv)[NT]) {
        const int x = 4 * s + krow;
        const bool second = x >= Ho;
        const int px = second ? x - Ho : x;
        const float* dl = second ? dl1 : dl0;
#pragma unroll
        for (int i = 0; i < MT; ++i) av[i] = img[(second ? abase1[i] : abase0[i]) + px * astep[i]];
#pragma unroll
        for (int j = 0; j < NT; ++j) bv[j] = dl[px * dstride + j * 16 + kcol];
    };
    auto mma = [&](const float (&av)[MT], const float (&bv)[NT]) {
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int j = 0; j < NT; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i], bv[j], acc[i][j], 0, 0, 0);
    };
    rd(0, a0, b0);
    for (int s = 0; s < nk; s += 2) {
        rd(s + 1, a1, b1);   // s + 1 <= nk: the second row's padding (zero dout) / finite LDS
        __builtin_amdgcn_sched_barrier(0);
        mma(a0, b0);
        __builtin_amdgcn_sched_barrier(0);
        if (s + 1 >= nk) break;
        rd(s + 2, a0, b0);
        __builtin_amdgcn_sched_barrier(0);
        mma(a1, b1);
        __builtin_amdgcn_sched_barrier(0);
    }
}

// MT = the m-tiles every wave of this launch runs (the plan buckets m-groups by
// ceil(tiles / 8)): a single loop body keeps the kernel at <= 128 VGPRs, i.e. two
// 8-wave workgroups per CU.  A wave with fewer real tiles multiplies the constant
// zero row for the rest (never written back).
// RPB = output rows per barrier.  1: the r03 schedule (input row y+k+1 and dout row
// y+2 issued at row y, a counted vmcnt keeps them in flight over the barrier).  2 (r06):
// rows y, y+1 between barriers, the next pair's two input rows and two dout rows
// issued before them and retired (vmcnt(0)) after them -- half the barriers, one
// more ring slot and dout buffer.  The same MFMAs per row in the same order: the
// same bits either way.  Measured (profiles/r06/wgrpb_sweep_*.log): 320 members
// 37.17 -> 37.06 ms per step, 40 members 5.58 -> 5.52 ms; the default is 2.
template <int OP, int NT, int MT, int RPB>
__global__ __launch_bounds__(kWgThreads) void conv_wgrad_kernel(StepArgs a, const WgItem* __restrict__ items) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const WgItem it = items[blockIdx.x];
    const Member& mb = a.mem[it.member];
    const int k = mb.k, F = mb.F;
    int Hin, Cin, Ho;
    long long dout_off, part_off;
    if (OP == WG_CONV1) {
        Hin = kImg; Cin = 1; Ho = mb.H1; dout_off = mb.dz1; part_off = mb.wp1;
    } else {
        Hin = mb.H1; Cin = F; Ho = mb.H2; dout_off = mb.dz2; part_off = mb.wp2;
    }
    const int N = F;
    const int Kw = k * k * Cin;
    const int RS = k + 1 + RPB;                 // ring slots
    const int rowf = Hin * Cin;                 // floats per input row
    const int rowS = round64(rowf);             // slot stride (a DMA chunk never crosses a slot)
    const int dcnt = Ho * N;                    // floats per dout row (pixel stride N)
    const int nk4 = (Ho + 3) >> 2;
    const int dS = round64((4 * nk4 + 4) * N + 64);   // dout buffer stride: zero padding past Ho*N
    float* ring = smem;                                              // [RS][rowS] (+ slack)
    const int ring_elems = RS * rowS + 8 * Cin + 64;                 // k-step padding reads stay in bounds
    constexpr int ND = 2 + RPB;                                      // dout row buffers
    float* dl = smem + round64(ring_elems);                          // [ND][dS]
    const int lds_floats = round64(ring_elems) + ND * dS;            // + kWgWaves*64 scratch, + {0, 1}
    const int kZero = lds_floats + kWgWaves * 64, kOne = kZero + 1;  // constant A rows (padding / bias)
    const float* zero_src = a.act + a.zero_off;                      // 64 zero floats in global memory
    const float* in_base = OP == WG_CONV1 ? a.x : a.act + mb.a1;
    const float* dout_base = a.act + dout_off;
    const int* order = a.order + (long long)it.member * a.order_stride + a.row0;

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int krow = lane >> 4, kcol = lane & 15;
    const int mtiles = (Kw + 1 + 15) >> 4;
    const int t0 = it.mg * (kWgRows / 16);
    const int mine = __builtin_amdgcn_readfirstlane(
        min(kWgMaxMT, max(0, (mtiles - t0 - wave + kWgWaves - 1) / kWgWaves)));

    // per lane, per tile: A row (ky, kx*Cin + c) -> ring address ring_row(y+ky)*rowS + col + x*Cin;
    // rows past Kw read the constant 0 (padding) or 1 (the bias row) with x stride 0
    int tky[MT], tcol[MT], astep[MT];
#pragma unroll
    for (int i = 0; i < MT; ++i) {
        const int m = (t0 + wave + kWgWaves * i) * 16 + (lane & 15);
        int ky = 0, col = m == Kw ? kOne : kZero, st = 0;
        if (m < Kw) {
            const int kc = k * Cin;
            ky = m / kc;
            col = m - ky * kc;
            st = Cin;
        }
        tky[i] = ky;
        tcol[i] = col;
        astep[i] = st;
    }
    f32x4 acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // zero all LDS once (ring slack, dout padding) before any DMA lands; the bias constant 1
    for (int e = tid; e <= kOne; e += kWgThreads) smem[e] = e == kOne ? 1.f : 0.f;
    __syncthreads();

    // kWgChunks DMA instructions: cnt floats of src -> LDS dst (64-float chunks, chunk q*8+wave)
    auto dma = [&](const float* src, int cnt, float* dst) {
#pragma unroll
        for (int q = 0; q < kWgChunks; ++q) {
            const int c0 = (q * kWgWaves + wave) * 64;
            const int e = c0 + lane;
            const float* g = e < cnt ? src + e : zero_src + lane;
            // chunks wholly past the row land in the scratch tail
            float* d = c0 < cnt ? dst + c0 : smem + lds_floats + wave * 64;
            __builtin_amdgcn_global_load_lds(g, (lds_ptr_t)d, 4, 0, 0);
        }
    };

    for (int b = it.b0; b < it.b1; ++b) {
        const float* inb = OP == WG_CONV1 ? in_base + (long long)order[b] * (kImg * kImg)
                                          : in_base + (long long)b * Hin * rowf;
        const float* dob = dout_base + (long long)b * Ho * dcnt;
        // prologue of the sample: input rows 0..k (slots 0..k), dout rows 0, 1
        for (int r = 0; r <= k && r < Hin; ++r) dma(inb + r * rowf, rowf, ring + r * rowS);
        dma(dob, dcnt, dl);
        if (Ho > 1) dma(dob + dcnt, dcnt, dl + dS);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        int slot0 = 0;   // ring slot of input row y
        if constexpr (RPB == 2) {
            for (int y = 0; y < Ho; y += 2) {
                // the next pair's rows: input rows y+k+1, y+k+2 -> the slots rows y-2, y-1
                // used; dout rows y+2, y+3 -> the buffers of dout rows y-2, y-1
                if (y + 2 < Ho) {
                    int sl = slot0 + k + 1;
                    sl = sl >= RS ? sl - RS : sl;
                    dma(inb + (y + k + 1) * rowf, rowf, ring + sl * rowS);
                    dma(dob + (y + 2) * dcnt, dcnt, dl + ((y + 2) & 3) * dS);
                    if (y + 3 < Ho) {
                        sl = sl + 1 == RS ? 0 : sl + 1;
                        dma(inb + (y + k + 2) * rowf, rowf, ring + sl * rowS);
                        dma(dob + (y + 3) * dcnt, dcnt, dl + ((y + 3) & 3) * dS);
                    }
                }
                if (a.wgpair && (Ho & 3) == 2) {   // Ho even here (H2 = 30 - 2k): pairs are whole
                    int ab0[MT], ab1[MT];
#pragma unroll
                    for (int i = 0; i < MT; ++i) {
                        int sl = slot0 + tky[i];
                        sl = sl >= RS ? sl - RS : sl;
                        ab0[i] = astep[i] ? sl * rowS + tcol[i] : tcol[i];
                        sl = sl + 1 == RS ? 0 : sl + 1;
                        ab1[i] = astep[i] ? sl * rowS + tcol[i] : tcol[i];
                    }
                    if (a.debug != 1 && mine > 0)
                        wgrad_row_pair<MT, NT>(ring, dl + (y & 3) * dS, dl + ((y + 1) & 3) * dS, ab0, ab1, astep, N, Ho,
                                               Ho >> 1, krow, kcol, acc);
                } else
#pragma unroll
                for (int dy = 0; dy < 2; ++dy) {
                    if (y + dy >= Ho) break;
                    int abase[MT];
#pragma unroll
                    for (int i = 0; i < MT; ++i) {
                        int sl = slot0 + dy + tky[i];
                        sl = sl >= RS ? sl - RS : sl;
                        abase[i] = astep[i] ? sl * rowS + tcol[i] : tcol[i];
                    }
                    const float* dcur = dl + ((y + dy) & 3) * dS;
                    if (a.debug != 1 && mine > 0) wgrad_row<MT, NT>(ring, dcur, abase, astep, N, nk4, krow, kcol, acc);
                }
                slot0 += 2;
                slot0 = slot0 >= RS ? slot0 - RS : slot0;
                asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
            }
            continue;
        }
        for (int y = 0; y < Ho; ++y) {
            // two rows ahead: input row y+k+1 -> the slot row y-1 used; dout row y+2
            const bool ahead = y + 2 < Ho;   // then input row y + k + 1 = (y + 2) + k - 1 < Hin too
            if (ahead) {
                int sl = slot0 + k + 1;
                sl = sl >= RS ? sl - RS : sl;
                dma(inb + (y + k + 1) * rowf, rowf, ring + sl * rowS);
                dma(dob + (y + 2) * dcnt, dcnt, dl + ((y + 2) % 3) * dS);
            }
            int abase[MT];
#pragma unroll
            for (int i = 0; i < MT; ++i) {
                int sl = slot0 + tky[i];
                sl = sl >= RS ? sl - RS : sl;
                abase[i] = astep[i] ? sl * rowS + tcol[i] : tcol[i];
            }
            const float* dcur = dl + (y % 3) * dS;
            if (a.debug != 1 && mine > 0) wgrad_row<MT, NT>(ring, dcur, abase, astep, N, nk4, krow, kcol, acc);
            slot0 = slot0 + 1 == RS ? 0 : slot0 + 1;
            // retire the DMA issued one row ago (row y+1's data); this row's stays in flight
            if (ahead) asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
        }
    }
    float* part = a.act + part_off + (long long)it.group * (Kw + 1) * N;
#pragma unroll
    for (int i = 0; i < MT; ++i) {
        if (i >= mine) break;
        const int mt = t0 + wave + kWgWaves * i;
#pragma unroll
        for (int j = 0; j < NT; ++j) {
            const int n = j * 16 + kcol;
            if (n >= N) continue;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = mt * 16 + krow * 4 + r;
                if (m <= Kw) part[(long long)m * N + n] = acc[i][j][r];
            }
        }
    }
}

// conv1 weight gradient (Cin = 1): M = k*k + 1 rows (the last one the bias), N = F,
// K = pixels.  M is at most 7 tiles, so the 8-wave m-group kernel above leaves most
// of its waves idle behind a barrier per output row.  Here every wave holds every
// m-tile of the member (MT = 1, 2, 4 or 7; padding tiles multiply the constant zero
// row) and the 4 waves split the K dimension: wave w takes output rows w, w+4, ...
// of the sample group's row stream.  The group's input images are staged in LDS
// once (one barrier); B fragments come straight from memory one row ahead.  The 4
// partial accumulators are summed through LDS in wave order (deterministic), into
// the same partial slab as conv_wgrad<WG_CONV1>.
constexpr int kW1Waves = 4;
constexpr int kW1Slack = 64;   // zero floats past the last image (padded k-steps)

__host__ __device__ constexpr inline int w1_lds_floats(int nb, int mt, int nt) {
    return (nb * kImg * kImg + kW1Slack + 2) > (mt * nt * 4 * 64) ? (nb * kImg * kImg + kW1Slack + 2)
                                                                  : (mt * nt * 4 * 64);
}

template <int NT, int MT>
__global__ __launch_bounds__(kW1Waves * 64) void conv1_wgrad_kernel(StepArgs a, const WgItem* __restrict__ items) {
    extern __shared__ __attribute__((aligned(16))) float sh[];   // images | slack | {0, 1}; then the reduction
    const WgItem it = items[blockIdx.x];
    const Member& mb = a.mem[it.member];
    const int k = mb.k, F = mb.F, Ho = mb.H1, Kw = k * k;
    const int tid = threadIdx.x, lane = tid & 63, krow = lane >> 4, kcol = lane & 15;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nk4 = (Ho + 3) >> 2;   // <= 7 (Ho <= 27)
    const int nb = it.b1 - it.b0, nrows = nb * Ho;
    const int kC0 = nb * kImg * kImg + kW1Slack, kC1 = kC0 + 1;
    const int* order = a.order + (long long)it.member * a.order_stride + a.row0;
    const float* zero = a.act + a.zero_off;
    const float* dz1 = a.act + mb.dz1;

    // stage the group's images (the k-fold index gather happens here)
    for (int bl = 0; bl < nb; ++bl) {
        const float* src = a.x + (long long)order[it.b0 + bl] * (kImg * kImg);
        for (int e = tid; e < kImg * kImg; e += kW1Waves * 64) sh[bl * kImg * kImg + e] = src[e];
    }
    for (int e = nb * kImg * kImg + tid; e <= kC1; e += kW1Waves * 64) sh[e] = e == kC1 ? 1.f : 0.f;

    int aoff[MT], ast[MT];
#pragma unroll
    for (int i = 0; i < MT; ++i) {
        const int m = i * 16 + (lane & 15);
        if (m < Kw) {
            const int ky = m / k, kx = m - ky * k;
            aoff[i] = ky * kImg + kx;
            ast[i] = 1;
        } else {
            aoff[i] = m == Kw ? kC1 : kC0;
            ast[i] = 0;
        }
    }
    // B fragments of dout row r (sample it.b0 + r / Ho): pixel 4s + krow, channel 16j + kcol;
    // past the row, the channels or the stream they read zeros
    auto loadB = [&](int r, float (&dst)[7][NT]) {
        const int bl = r / Ho, y = r - bl * Ho;
        const float* row = dz1 + ((long long)(it.b0 + bl) * Ho + y) * Ho * F;
#pragma unroll
        for (int s = 0; s < 7; ++s) {
            const int x = 4 * s + krow;
#pragma unroll
            for (int j = 0; j < NT; ++j) {
                const int n = j * 16 + kcol;
                const bool ok = r < nrows && s < nk4 && x < Ho && n < F;
                dst[s][j] = *(ok ? row + x * F + n : zero + lane);
            }
        }
    };
    f32x4 acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto row = [&](int r, const float (&bq)[7][NT]) {
        const int bl = r / Ho, y = r - bl * Ho;
        int ab[MT];
#pragma unroll
        for (int i = 0; i < MT; ++i) ab[i] = ast[i] ? aoff[i] + bl * kImg * kImg + y * kImg : aoff[i];
#pragma unroll
        for (int s = 0; s < 7; ++s) {
            if (s >= nk4) break;
            const int x = 4 * s + krow;
            float av[MT];
#pragma unroll
            for (int i = 0; i < MT; ++i) av[i] = sh[ab[i] + x * ast[i]];
#pragma unroll
            for (int i = 0; i < MT; ++i)
#pragma unroll
                for (int j = 0; j < NT; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i], bq[s][j], acc[i][j], 0, 0, 0);
        }
    };

    float b0[7][NT], b1[7][NT];
    loadB(wave, b0);
    __syncthreads();
    if (a.debug != 1) {
        for (int r = wave; r < nrows; r += 2 * kW1Waves) {
            loadB(r + kW1Waves, b1);
            row(r, b0);
            if (r + kW1Waves >= nrows) break;
            loadB(r + 2 * kW1Waves, b0);
            row(r + kW1Waves, b1);
        }
    }

    // fixed-order cross-wave sum through LDS (reusing the image space), then the slab
    __syncthreads();
    for (int w = 0; w < kW1Waves; ++w) {
        if (wave == w) {
#pragma unroll
            for (int i = 0; i < MT; ++i)
#pragma unroll
                for (int j = 0; j < NT; ++j)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        float* q = sh + ((i * NT + j) * 4 + r) * 64 + lane;
                        const float v = w == 0 ? acc[i][j][r] : *q + acc[i][j][r];
                        if (w + 1 < kW1Waves) *q = v; else acc[i][j][r] = v;
                    }
        }
        if (w + 1 < kW1Waves) __syncthreads();
    }
    if (wave != kW1Waves - 1) return;
    float* part = a.act + mb.wp1 + (long long)it.group * (Kw + 1) * F;
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) {
            const int n = j * 16 + kcol;
            if (n >= F) continue;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = i * 16 + krow * 4 + r;
                if (m <= Kw) part[(long long)m * F + n] = acc[i][j][r];
            }
        }
}

// Sum the per-group partial slabs (fixed order) into the weight gradients.
__global__ void wgrad_reduce_kernel(StepArgs a, const MItem* __restrict__ items, int per_block) {
    const MItem it = items[blockIdx.y];
    const Member& mb = a.mem[it.member];
    const int conv = it.aux;  // 0 conv1, 1 conv2
    const long long Sw = conv ? (long long)mb.k * mb.k * mb.F * mb.F : (long long)mb.k * mb.k * mb.F;
    const long long S = Sw + mb.F;   // weight rows + the bias row
    const int G = conv ? mb.g2 : mb.g1;
    const float* part = a.act + (conv ? mb.wp2 : mb.wp1);
    float* gw = a.grads + (conv ? mb.w2 : mb.w1);
    float* gb = a.grads + (conv ? mb.b2 : mb.b1);
    for (long long i = (long long)blockIdx.x * per_block + threadIdx.x; i < S && i < (long long)(blockIdx.x + 1) * per_block;
         i += blockDim.x) {
        // slabs summed in slab order; loads issued 8 at a time ahead of the adds
        float s = 0.f;
        int q = 0;
        for (; q + 8 <= G; q += 8) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = part[(q + u) * S + i];
#pragma unroll
            for (int u = 0; u < 8; ++u) s += v[u];
        }
        for (; q < G; ++q) s += part[q * S + i];
        if (i < Sw) gw[i] = s; else gb[i - Sw] = s;
    }
}

// w2t[(ky', kx')][f][c] = w2[(k-1-ky', k-1-kx', c)][f]: weights of the input-gradient
// conv, zero-padded to [k*k][F4][16*NT] so every dgrad fragment load is in bounds.
__global__ void flip_w2_kernel(StepArgs a, const MItem* __restrict__ items) {
    const Member& mb = a.mem[items[blockIdx.y].member];
    const int k = mb.k, F = mb.F;
    const int F4 = (F + 3) & ~3, N16 = mb.nt * 16;
    const long long S = (long long)k * k * F4 * N16;
    const float* w2 = a.params + mb.w2;
    float* w2t = a.act + mb.w2t;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < S; i += (long long)gridDim.x * blockDim.x) {
        const int c = i % N16;
        const long long r = i / N16;
        const int f = r % F4;
        const int tap = r / F4;
        const int ky = tap / k, kx = tap % k;
        const int src_tap = (k - 1 - ky) * k + (k - 1 - kx);
        w2t[i] = (f < F && c < F) ? w2[((long long)src_tap * F + c) * F + f] : 0.f;
    }
    // forward weights, zero-padded to [K16 + kWSlack][N16]
    const int K2 = k * k * F, K1 = k * k;
    const long long S2 = (long long)(((K2 + 15) & ~15) + kWSlack) * N16;
    const long long S1 = (long long)(((K1 + 15) & ~15) + kWSlack) * N16;
    float* w2p = a.act + mb.w2p;
    float* w1p = a.act + mb.w1p;
    const float* w1 = a.params + mb.w1;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < S2; i += (long long)gridDim.x * blockDim.x) {
        const int c = i % N16;
        const long long r = i / N16;
        w2p[i] = (r < K2 && c < F) ? w2[r * F + c] : 0.f;
    }
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < S1; i += (long long)gridDim.x * blockDim.x) {
        const int c = i % N16;
        const long long r = i / N16;
        w1p[i] = (r < K1 && c < F) ? w1[r * F + c] : 0.f;
    }
}

// ============================================================================
// Max-pool (floor mode, stride p) + dropout, and its backward.
// ============================================================================
__global__ __launch_bounds__(256) void pool_fwd_kernel(StepArgs a, const MItem* __restrict__ items) {
    const MItem it = items[blockIdx.x];
    const Member& mb = a.mem[it.member];
    const int b = it.aux;
    const int F = mb.F, p = mb.p, s = mb.s, H2 = mb.H2, K1 = mb.K1;
    const float* a2 = a.act + mb.a2 + (long long)b * H2 * H2 * F;
    float* pd = a.act + mb.pd + (long long)b * K1;
    unsigned char* am = reinterpret_cast<unsigned char*>(a.act + mb.am) + (long long)b * K1;
    const unsigned base = drop_base(mb.seed, a.step, 0);
    for (int j = threadIdx.x; j < K1; j += blockDim.x) {
        const int f = j % F, q = j / F;
        const int px = q % s, py = q / s;
        float best = -__builtin_huge_valf();
        int arg = 0;
        for (int dy = 0; dy < p; ++dy)
            for (int dx = 0; dx < p; ++dx) {
                const float v = a2[((py * p + dy) * H2 + (px * p + dx)) * F + f];
                if (v > best) { best = v; arg = dy * p + dx; }
            }
        float o = best;
        if (a.train) o = drop_keep(base, (unsigned)(b * K1 + j), mb.drop_thr) ? best * mb.inv_keep : 0.f;
        pd[j] = o;
        am[j] = (unsigned char)arg;
    }
}

__global__ __launch_bounds__(256) void pool_bwd_kernel(StepArgs a, const MItem* __restrict__ items) {
    const MItem it = items[blockIdx.x];
    const Member& mb = a.mem[it.member];
    const int b = it.aux;
    const int F = mb.F, p = mb.p, s = mb.s, H2 = mb.H2, K1 = mb.K1;
    const float* a2 = a.act + mb.a2 + (long long)b * H2 * H2 * F;
    const float* dp = a.act + mb.dp + (long long)b * K1;
    const unsigned char* am = reinterpret_cast<const unsigned char*>(a.act + mb.am) + (long long)b * K1;
    float* dz2 = a.act + mb.dz2 + (long long)b * H2 * H2 * F;
    const int n = H2 * H2 * F;
    // division-free walk over (y, x, f): each thread advances by blockDim.x elements
    const float inv_p = 1.f / (float)p;   // floor((x + 0.5) / p) is exact for x < 64, p <= 13
    const int step = blockDim.x, df = step % F, dq = step / F;
    int f = threadIdx.x % F, q = threadIdx.x / F;
    int x = q % H2, y = q / H2;
    for (int e = threadIdx.x; e < n; e += step) {
        const int py = (int)(((float)y + 0.5f) * inv_p), px = (int)(((float)x + 0.5f) * inv_p);
        float v = 0.f;
        if (py < s && px < s) {
            const int j = (py * s + px) * F + f;
            if (am[j] == (y - py * p) * p + (x - px * p)) v = dp[j];
        }
        dz2[e] = a2[e] > 0.f ? v : 0.f;
        f += df;
        x += dq;
        if (f >= F) { f -= F; ++x; }
        while (x >= H2) { x -= H2; ++y; }
    }
}

// ============================================================================
// Grouped dense GEMMs (MFMA f32 16x16x4), 64x64 tiles, 4 waves as 2x2 of 32x32;
// K in chunks of 32, the next chunk's global loads in flight during the MFMAs.
// ============================================================================
template <int OP>
struct DenseGeom {
    int M, N, K;
    const float* A; long long sai, sak;
    const float* Bm; long long sbk, sbj;
    float* C; long long ldc;
};

template <int OP>
__device__ __forceinline__ DenseGeom<OP> dense_geom(const StepArgs& a, const Member& mb) {
    DenseGeom<OP> g;
    const int B = a.B;
    const int K1 = mb.K1, D = mb.dense;
    if (OP == D1_FWD) {
        g.M = B; g.N = D; g.K = K1;
        g.A = a.act + mb.pd; g.sai = K1; g.sak = 1;
        g.Bm = a.params + mb.w3; g.sbk = D; g.sbj = 1;
        g.C = a.act + mb.h; g.ldc = D;
    } else if (OP == D2_FWD) {
        g.M = B; g.N = kClasses; g.K = D;
        g.A = a.act + mb.hd; g.sai = D; g.sak = 1;
        g.Bm = a.params + mb.w4; g.sbk = kClasses; g.sbj = 1;
        g.C = a.act + mb.z3; g.ldc = kClasses;
    } else if (OP == D2_WGRAD) {
        g.M = D; g.N = kClasses; g.K = B;
        g.A = a.act + mb.hd; g.sai = 1; g.sak = D;
        g.Bm = a.act + mb.dz3; g.sbk = kClasses; g.sbj = 1;
        g.C = a.grads + mb.w4; g.ldc = kClasses;
    } else if (OP == D2_DGRAD) {
        g.M = B; g.N = D; g.K = kClasses;
        g.A = a.act + mb.dz3; g.sai = kClasses; g.sak = 1;
        g.Bm = a.params + mb.w4; g.sbk = 1; g.sbj = kClasses;
        g.C = a.act + mb.dh; g.ldc = D;
    } else if (OP == D1_WGRAD) {
        g.M = K1; g.N = D; g.K = B;
        g.A = a.act + mb.pd; g.sai = 1; g.sak = K1;
        g.Bm = a.act + mb.dh; g.sbk = D; g.sbj = 1;
        g.C = a.grads + mb.w3; g.ldc = D;
    } else {  // D1_DGRAD
        g.M = B; g.N = K1; g.K = D;
        g.A = a.act + mb.dh; g.sai = D; g.sak = 1;
        g.Bm = a.params + mb.w3; g.sbk = 1; g.sbj = D;
        g.C = a.act + mb.dp; g.ldc = K1;
    }
    return g;
}

template <int OP>
__global__ __launch_bounds__(256) void dense_kernel(StepArgs a, const GemmItem* __restrict__ items) {
    constexpr int BM = 64, BN = 64, BK = 32;
    constexpr int EA = BM * BK / 256, EB = BN * BK / 256;   // staged elements per thread
    __shared__ float As[BK][BM + 1];
    __shared__ float Bs[BK][BN + 16];
    const GemmItem it = items[blockIdx.x];
    const Member& mb = a.mem[it.member];
    const DenseGeom<OP> g = dense_geom<OP>(a, mb);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave >> 1, wc = wave & 1;
    const int krow = lane >> 4, kcol = lane & 15;
    f32x4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // (i, kk) / (j, kk) of this thread's staged elements: fixed for the whole K loop
    auto a_ik = [&](int q, int& i, int& kk) {
        const int e = tid + 256 * q;
        if (g.sak == 1) { i = e / BK; kk = e % BK; } else { kk = e / BM; i = e % BM; }
    };
    auto b_jk = [&](int q, int& j, int& kk) {
        const int e = tid + 256 * q;
        if (g.sbj == 1) { kk = e / BN; j = e % BN; } else { j = e / BK; kk = e % BK; }
    };
    float ra[EA], rb[EB];
    auto load = [&](int k0) {   // global -> registers (chunk k0), in flight during the MFMAs
#pragma unroll
        for (int q = 0; q < EA; ++q) {
            int i, kk;
            a_ik(q, i, kk);
            const int gi = it.m0 + i, gk = k0 + kk;
            ra[q] = (gi < g.M && gk < g.K) ? g.A[gi * g.sai + gk * g.sak] : 0.f;
        }
#pragma unroll
        for (int q = 0; q < EB; ++q) {
            int j, kk;
            b_jk(q, j, kk);
            const int gj = it.n0 + j, gk = k0 + kk;
            rb[q] = (gj < g.N && gk < g.K) ? g.Bm[gk * g.sbk + gj * g.sbj] : 0.f;
        }
    };
    load(0);
    for (int k0 = 0; k0 < g.K; k0 += BK) {
#pragma unroll
        for (int q = 0; q < EA; ++q) {
            int i, kk;
            a_ik(q, i, kk);
            As[kk][i] = ra[q];
        }
#pragma unroll
        for (int q = 0; q < EB; ++q) {
            int j, kk;
            b_jk(q, j, kk);
            Bs[kk][j] = rb[q];
        }
        __syncthreads();
        if (k0 + BK < g.K) load(k0 + BK);
#pragma unroll
        for (int ks = 0; ks < BK; ks += 4) {
            float af[2], bf[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) af[i] = As[ks + krow][wr * 32 + i * 16 + kcol];
#pragma unroll
            for (int j = 0; j < 2; ++j) bf[j] = Bs[ks + krow][wc * 32 + j * 16 + kcol];
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bf[j], acc[i][j], 0, 0, 0);
        }
        __syncthreads();
    }
    const unsigned base1 = drop_base(mb.seed, a.step, 1);
    const unsigned base0 = drop_base(mb.seed, a.step, 0);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int gi = it.m0 + wr * 32 + i * 16 + krow * 4 + r;
                const int gj = it.n0 + wc * 32 + j * 16 + kcol;
                if (gi >= g.M || gj >= g.N) continue;
                float v = acc[i][j][r];
                const long long o = (long long)gi * g.ldc + gj;
                if (OP == D1_FWD) {
                    v = fmaxf(v + a.params[mb.b3 + gj], 0.f);
                    g.C[o] = v;
                    float hd = v;
                    if (a.train) hd = drop_keep(base1, (unsigned)o, mb.drop_thr) ? v * mb.inv_keep : 0.f;
                    a.act[mb.hd + o] = hd;
                } else if (OP == D2_FWD) {
                    g.C[o] = v + a.params[mb.b4 + gj];
                } else if (OP == D2_DGRAD) {
                    const bool keep = drop_keep(base1, (unsigned)o, mb.drop_thr);
                    g.C[o] = (keep && a.act[mb.h + o] > 0.f) ? v * mb.inv_keep : 0.f;
                } else if (OP == D1_DGRAD) {
                    g.C[o] = drop_keep(base0, (unsigned)o, mb.drop_thr) ? v * mb.inv_keep : 0.f;
                } else {
                    g.C[o] = v;
                }
            }
}

// ============================================================================
// softmax + Keras binary_crossentropy (clip 1e-7, mean over classes and batch)
// One workgroup per member; one thread per sample row.
// ============================================================================
__global__ __launch_bounds__(256) void softmax_bce_kernel(StepArgs a, const MItem* __restrict__ items) {
    __shared__ float red[256];
    __shared__ int redc[256];
    const int member = items[blockIdx.x].member;
    const Member& mb = a.mem[member];
    const int B = a.B;
    const int tid = threadIdx.x;
    float lsum = 0.f;
    int corr = 0;
    for (int b = tid; b < B; b += 256) {
        const float* z = a.act + mb.z3 + (long long)b * kClasses;
        const int sidx = a.order[(long long)member * a.order_stride + a.row0 + b];
        const int y = a.labels[sidx];
        float zm = z[0];
        int am = 0;
#pragma unroll
        for (int c = 1; c < kClasses; ++c) if (z[c] > zm) { zm = z[c]; am = c; }
        float e[kClasses], s = 0.f;
#pragma unroll
        for (int c = 0; c < kClasses; ++c) { e[c] = expf(z[c] - zm); s += e[c]; }
        corr += (am == y);
        if (mb.loss == MPO_LOSS_CCE) {
            // Keras categorical_crossentropy: q = p / sum p, clipped target probability;
            // d loss / d logits = live (q - onehot) / B (the DenseNet head's form)
            float q[kClasses], S2 = 0.f;
#pragma unroll
            for (int c = 0; c < kClasses; ++c) { q[c] = e[c] / s; S2 += q[c]; }
#pragma unroll
            for (int c = 0; c < kClasses; ++c) q[c] /= S2;
            const float qt = q[y];
            lsum += -logf(fminf(fmaxf(qt, kBceEps), 1.f - kBceEps));
            if (a.train) {
                const float live = (qt >= kBceEps && qt <= 1.f - kBceEps) ? 1.f / (float)B : 0.f;
                float* dz = a.act + mb.dz3 + (long long)b * kClasses;
#pragma unroll
                for (int c = 0; c < kClasses; ++c) dz[c] = live * (q[c] - (c == y ? 1.f : 0.f));
            }
            continue;
        }
        float l = 0.f, gdot = 0.f, gp[kClasses], pr[kClasses];
#pragma unroll
        for (int c = 0; c < kClasses; ++c) {
            const float p = e[c] / s;
            pr[c] = p;
            const float t = (c == y) ? 1.f : 0.f;
            const float pc = fminf(fmaxf(p, kBceEps), 1.f - kBceEps);
            l += -(t * logf(pc) + (1.f - t) * logf(1.f - pc));
            const bool inside = p > kBceEps && p < 1.f - kBceEps;
            gp[c] = inside ? (pc - t) / (pc * (1.f - pc)) / (float)(kClasses * B) : 0.f;
            gdot += gp[c] * p;
        }
        lsum += l / (float)kClasses;
        if (a.train) {
            float* dz = a.act + mb.dz3 + (long long)b * kClasses;
#pragma unroll
            for (int c = 0; c < kClasses; ++c) dz[c] = pr[c] * (gp[c] - gdot);
        }
    }
    red[tid] = lsum;
    redc[tid] = corr;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (tid < s) { red[tid] += red[tid + s]; redc[tid] += redc[tid + s]; }
        __syncthreads();
    }
    if (tid == 0) {
        if (a.train) {
            a.loss_out[member] = red[0] / (float)B;
        } else {
            a.loss_sum[member] += red[0];
            a.correct[member] += redc[0];
        }
    }
}

// ============================================================================
// Bias gradients: column sums of dz1 / dz2 / dh / dz3 (deterministic).
// item.aux: 0 b1 (dz1, B*H1^2 x F), 1 b2 (dz2, B*H2^2 x F), 2 b3 (dh, B x dense), 3 b4 (dz3, B x 10)
// ============================================================================
__global__ __launch_bounds__(256) void colsum_kernel(StepArgs a, const MItem* __restrict__ items) {
    __shared__ float red[4][64];
    const MItem it = items[blockIdx.x];
    const Member& mb = a.mem[it.member];
    const int B = a.B;
    const float* src;
    long long rows;
    int N;
    float* dst;
    if (it.aux == 0) { src = a.act + mb.dz1; rows = (long long)B * mb.H1 * mb.H1; N = mb.F; dst = a.grads + mb.b1; }
    else if (it.aux == 1) { src = a.act + mb.dz2; rows = (long long)B * mb.H2 * mb.H2; N = mb.F; dst = a.grads + mb.b2; }
    else if (it.aux == 2) { src = a.act + mb.dh; rows = B; N = mb.dense; dst = a.grads + mb.b3; }
    else { src = a.act + mb.dz3; rows = B; N = kClasses; dst = a.grads + mb.b4; }
    const int tid = threadIdx.x;
    const int rl = tid >> 6, cl = tid & 63;
    for (int c0 = 0; c0 < N; c0 += 64) {
        const int c = c0 + cl;
        float s = 0.f;
        if (c < N)
            for (long long r = rl; r < rows; r += 4) s += src[r * N + c];
        red[rl][cl] = s;
        __syncthreads();
        if (rl == 0 && c < N) dst[c] = (red[0][cl] + red[1][cl]) + (red[2][cl] + red[3][cl]);
        __syncthreads();
    }
}

// ============================================================================
// Adam (Keras form): lr_t = lr sqrt(1-b2^t)/(1-b1^t); p -= lr_t m / (sqrt(v) + eps)
// ============================================================================
__global__ __launch_bounds__(256) void adam_kernel(StepArgs a, const MItem* __restrict__ items, float* __restrict__ params,
                                                   float* __restrict__ mo, float* __restrict__ vo, int t, float b1,
                                                   float b2, float eps, int chunk) {
    const MItem it = items[blockIdx.x];
    const Member& mb = a.mem[it.member];
    const long long begin = mb.w1 + (long long)it.aux * chunk;
    const long long end = min(mb.pend, begin + chunk);
    if (mb.opt == MPO_OPT_SGD) {            // Keras SGD, no momentum
        for (long long i = begin + threadIdx.x; i < end; i += blockDim.x) params[i] -= mb.lr * a.grads[i];
        return;
    }
    const double corr = sqrt(1.0 - pow((double)b2, t)) / (1.0 - pow((double)b1, t));
    const float lr_t = (float)(mb.lr * corr);
    for (long long i = begin + threadIdx.x; i < end; i += blockDim.x) {
        const float g = a.grads[i];
        const float m = b1 * mo[i] + (1.f - b1) * g;
        const float v = b2 * vo[i] + (1.f - b2) * g * g;
        mo[i] = m;
        vo[i] = v;
        params[i] -= lr_t * m / (sqrtf(v) + eps);
    }
}

__global__ void kfold_gather_kernel(const float* __restrict__ X, const int* __restrict__ idx, long long rows, int row_elems,
                                    float* __restrict__ out) {
    const long long r = blockIdx.y + (long long)blockIdx.z * 65535;
    if (r >= rows) return;
    const float* src = X + (long long)idx[r] * row_elems;
    float* dst = out + r * row_elems;
    for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < row_elems; e += gridDim.x * blockDim.x) dst[e] = src[e];
}

// ============================================================================
// Host-side plan
// ============================================================================
// Launch segments of one op: items sorted by (NT, occupancy class), one launch
// per segment with that segment's own dynamic LDS size.  Bucketing by NT alone
// would size every block of a bucket for its largest member and cap the whole
// bucket at that member's occupancy.
struct Seg {
    int nt, begin, end;
    size_t lds;
    int sub;   // wgrad: m-tiles per wave (WgItem::R); 0 for the other ops
};
inline int item_sub(const WgItem& x) { return x.R; }
template <class T>
inline int item_sub(const T&) { return 0; }
struct Bucketed {
    std::vector<Seg> segs;
};

// Per-phase device timing for diagnostics (env MPO_POP_PROFILE=1 at plan
// creation): hipEvents between the launches of a step, accumulated on the host
// after an event sync.  Off by default (no events, no syncs).
struct PhaseTimer {
    bool on = false;
    std::vector<hipEvent_t> ev;
    std::vector<std::string> names;
    int used = 0;
    std::vector<std::pair<std::string, double>> acc;
    void mark(const std::string& name, hipStream_t s) {
        if (!on) return;
        if (used == (int)ev.size()) {
            hipEvent_t e;
            if (hipEventCreate(&e) != hipSuccess) { on = false; return; }
            ev.push_back(e);
            names.emplace_back();
        }
        names[used] = name;
        (void)hipEventRecord(ev[used], s);
        ++used;
    }
    void finish() {
        if (!on || used < 2) { used = 0; return; }
        (void)hipEventSynchronize(ev[used - 1]);
        for (int i = 1; i < used; ++i) {
            float ms = 0.f;
            (void)hipEventElapsedTime(&ms, ev[i - 1], ev[i]);
            auto it = std::find_if(acc.begin(), acc.end(), [&](const auto& p) { return p.first == names[i]; });
            if (it == acc.end()) acc.emplace_back(names[i], (double)ms); else it->second += ms;
        }
        used = 0;
    }
    ~PhaseTimer() { for (auto e : ev) (void)hipEventDestroy(e); }
};

// Integer tuning knob from the environment (read once per plan; A/B only).
int env_int(const char* name, int dflt) {
    const char* v = getenv(name);
    return (v && *v) ? atoi(v) : dflt;
}

// Planner overrides for tuning sweeps, one variable: MPO_POP_PLAN="key=value,..."
// (keys: wgrpb = 1 | 2, wgs = 1 | 2, dgs = 2 | 3, dbg = MPO_POP_DEBUG, xcd = items per XCD run (0: plain order), dg_tiles, dg_kb, conv_mt, conv_kb1, conv_kb2, wg_spg1, wg_spg2, streams = 1 | 2 | 3,
// occmerge = 0 | 1 | 2, occfill = quarter waves, see bucket_segs).  Every
// value only changes how work is cut into items or ordered over streams, never the arithmetic.
int plan_knob(const char* key, int dflt) {
    const char* v = getenv("MPO_POP_PLAN");
    if (!v) return dflt;
    const size_t n = strlen(key);
    for (const char* p = v; *p;) {
        if (!strncmp(p, key, n) && p[n] == '=') return atoi(p + n + 1);
        const char* c = strchr(p, ',');
        if (!c) break;
        p = c + 1;
    }
    return dflt;
}

struct Plan {
    int n = 0, B = 0;
    PhaseTimer timer;
    bool timer_detail = false;
    long long zero_off = 0;
    int debug = 0;
    std::vector<Member> mem;
    long long n_params = 0, act_floats = 0;
    std::vector<ConvItem> conv1, conv2, dgrad, dgf;
    Bucketed bc1, bc2, bdg, bdf;
    std::vector<WgItem> wg1, wg2;
    Bucketed bw1, bw2;
    std::vector<GemmItem> d1f, d2f, d2w, d2d, d1w, d1d;
    std::vector<MItem> per_member, per_sample, colsum, wred, adam;
    int adam_chunk = 8192;
    int wred_per_block = 4096, wred_blocks = 1;
    // device tables
    char* table_base = nullptr;
    size_t table_bytes = 0;
    std::vector<char> host_tables;
    size_t off_mem, off_conv1, off_conv2, off_dgrad, off_dgf, off_wg1, off_wg2, off_d1f, off_d2f, off_d2w, off_d2d,
        off_d1w, off_d1d, off_pm, off_ps, off_cs, off_wr, off_adam;
    float *params = nullptr, *grads = nullptr, *m = nullptr, *v = nullptr, *act = nullptr;
    bool bound = false;
    size_t lds_conv_max = 0, lds_wg_max = 0;
    int conv_mt = 4;        // forward conv m-tiles per wave at most: items of up to 256 pixels (MPO_POP_PLAN conv_mt=2: 128)
    int dg_tiles = 12;      // 4x4 tiles per conv2 input-gradient work item at most (MPO_POP_PLAN dg_tiles)
    int dgfset = 0;         // ... and members whose bit k is set (MPO_POP_PLAN dgfset, a mask over k)
    int dgfwd = 4;          // r06: members with k <= dgfwd take the zero-bordered forward conv for their input gradient (MPO_POP_PLAN dgfwd)
    int wgrpb = 2;          // conv2 weight gradient output rows per barrier (MPO_POP_PLAN wgrpb = 1 | 2)
    int wgpair = 1;         // r06: with wgrpb 2, a row pair of Ho = 2 (mod 4) pixels as one K run (MPO_POP_PLAN wgpair)
    // Second stream for independent launches (MPO_POP_PLAN streams=1 keeps one): the
    // forward conv2 buckets alternate between the two, and the conv2 weight gradient
    // runs beside the input gradient + conv1 weight gradient, so one launch's tail
    // overlaps the other's work.  No two concurrent kernels write the same buffer.
    mpo::SideStream side;
    mpo::SideStream side4;   // r06: a third stream for the input-gradient buckets (plan knob dgs = 3, the default; 2: two)
    mpo::SideStream side3;   // r06: conv2 weight-gradient buckets alternate over side and side3 (plan knob wgs = 2, the default; 1: one stream)
    mpo::SideStream side2;   // a third stream: the input-gradient buckets alternate over s and it
};

size_t conv_lds_bytes(int rows, int Wp, int Cin, int Ho, int K, int nt) {
    (void)nt;
    const int Fp = fwd_fp(Cin);
    (void)Fp;
    return (size_t)(align4(rows * fwd_rs(Wp, Cin, Ho)) + ((K + 15) & ~15) + kKoffSlack) * sizeof(float);
}

size_t dgrad_lds_bytes(int R, int k, int F, int H2) {
    const int rows = std::min(H2, R + k - 1);   // dz2 rows of the widest chunk (unpadded)
    return (size_t)(align4(rows * dgrad_rs(H2, F)) + 64) * sizeof(float);
}

size_t wg_lds_bytes(int k, int Hin, int Cin, int Ho, int F, int rpb = 1) {
    const int ring = round64((k + 1 + rpb) * round64(Hin * Cin) + 8 * Cin + 64);
    const int dS = round64((4 * ((Ho + 3) >> 2) + 4) * F + 64);
    return (size_t)(ring + (2 + rpb) * dS + kWgWaves * 64 + 4) * sizeof(float);
}

// Row-chunk height: as many output rows as fit M = R*Ho <= mcap pixels, shrunk
// (down to half of that) to fit the kb1 budget, else kb2, when possible (r03 plan: 256 pixels, 40 / 100 KiB).
template <class Fn>
int choose_rows(int Ho, Fn lds_of, int kb1 = 52, int kb2 = 78, int mcap = 128) {
    const int rmax = std::max(1, std::min(Ho, mcap / Ho));
    const int rmin = std::max(1, rmax / 2);
    for (size_t budget : {(size_t)kb1 << 10, (size_t)kb2 << 10})
        for (int R = rmax; R >= rmin; --R)
            if (lds_of(R) <= budget) return R;
    for (int R = rmax; R >= 1; --R)
        if (lds_of(R) <= ((size_t)160 << 10)) return R;
    return 1;
}

// Workgroups per CU that `lds` bytes allow (LDS 160 KiB; 8 = the 32-wave cap).
int lds_class(size_t lds) { return (int)std::min<size_t>(8, ((size_t)160 << 10) / std::max<size_t>(lds, 1)); }

// mode 0: one segment per (NT, sub, occupancy class); 1: one per (NT, sub) at the
// largest member's LDS; 2: adjacent occupancy classes of one (NT, sub) merge while
// either of them is short of one full wave of workgroups at its own occupancy
template <class T>
void bucket_segs(std::vector<T>& items, Bucketed& bk, const std::vector<Member>& mem, const std::vector<size_t>& lds,
                 int mode = 0) {
    const bool by_occupancy = mode != 1;
    // by_occupancy = false: one segment per (NT, sub) at the largest member's LDS (fewer, fuller launches)
    auto key = [&](const T& x) {
        return (mem[x.member].nt * 8 + item_sub(x)) * 16 + (by_occupancy ? 8 - lds_class(lds[x.member]) : 0);
    };
    std::stable_sort(items.begin(), items.end(), [&](const T& x, const T& y) { return key(x) < key(y); });
    bk.segs.clear();
    for (int i = 0; i < (int)items.size();) {
        const int kk = key(items[i]);
        Seg sg{mem[items[i].member].nt, i, i, 0, item_sub(items[i])};
        while (i < (int)items.size() && key(items[i]) == kk) {
            sg.lds = std::max(sg.lds, lds[items[i].member]);
            ++i;
        }
        sg.end = i;
        if (mode == 2 && !bk.segs.empty()) {
            Seg& pv = bk.segs.back();
            static const long long fill4 = std::max(1, plan_knob("occfill", 4));   // quarter waves
            const long long full_pv = 64LL * fill4 * lds_class(pv.lds), full_sg = 64LL * fill4 * lds_class(sg.lds);
            if (pv.nt == sg.nt && pv.sub == sg.sub &&
                (pv.end - pv.begin < full_pv || sg.end - sg.begin < full_sg)) {
                pv.end = sg.end;
                pv.lds = std::max(pv.lds, sg.lds);
                continue;
            }
        }
        bk.segs.push_back(sg);
    }
}

// XCD-aware order of a segment's work items (speed only: an item's arithmetic does not
// depend on the block that runs it, and nothing relies on where a block runs).  The
// dispatcher is observed to deal blocks round-robin over the 8 XCDs (blocks b and b + 8
// share an XCD and its 4 MiB L2; MI355X_MICROARCH.md, workgroup dispatch), while a
// segment's items are member-major: a sample's row chunks, a wgrad sample group's
// m-groups and a member's samples sit next to each other and re-read the same rows and
// weights.  Runs of `c` consecutive items are dealt whole to one XCD group (run t to
// group t % 8), so those re-reads meet in one L2; the runs stay interleaved over the
// groups, so every XCD still gets an even share of every member size (one contiguous
// eighth per XCD -- c = n / 8 -- measured 21% SLOWER on the 320-member step despite
// 16% less HBM traffic: the eighths' costs differ).  The table is stored permuted.
// r06, MI355X, 320 members (profiles/r06/xcd_*.log): runs of c = 4 items cut the
// measured HBM traffic per train batch 37.9 -> 33.8 GB (conv_wgrad 11.9 -> 8.7 GB, its
// m-groups' row re-reads now meet in one L2) for +0.3% step time (37.05 -> 37.16 ms;
// the kernels are issue-bound, not HBM-bound); c = 2 / 8 / 16 / 32: 37.2-37.4 ms.
// MPO_POP_PLAN xcd=0 restores the plain order.
template <class T>
void xcd_deal(std::vector<T>& items, const Bucketed& bk, int c) {
    if (c <= 1) return;
    std::vector<T> out;
    for (const Seg& sg : bk.segs) {
        const int n = sg.end - sg.begin;
        if (n <= 8) continue;
        std::vector<std::vector<int>> q(8);
        for (int i = 0; i < n; ++i) q[(i / c) & 7].push_back(i);
        // blocks b < n with b % 8 == x: n / 8 (+1 for x < n % 8); the surplus of the
        // groups that got the partial last runs moves to the groups short of blocks
        std::vector<int> spill;
        for (int x = 0; x < 8; ++x) {
            const size_t cap = n / 8 + (x < n % 8 ? 1 : 0);
            while (q[x].size() > cap) { spill.push_back(q[x].back()); q[x].pop_back(); }
        }
        for (int x = 0; x < 8; ++x) {
            const size_t cap = n / 8 + (x < n % 8 ? 1 : 0);
            while (q[x].size() < cap) { q[x].push_back(spill.back()); spill.pop_back(); }
        }
        out.assign(n, items[sg.begin]);
        for (int b = 0; b < n; ++b) out[b] = items[sg.begin + q[b & 7][b >> 3]];
        std::copy(out.begin(), out.end(), items.begin() + sg.begin);
    }
}

// m-tiles per wave of wgrad m-group mg for a GEMM of Kw + 1 rows (bias row included)
int wg_mt(int Kw, int mg) {
    const int mtiles = (Kw + 1 + 15) / 16;
    const int tiles = std::min(kWgRows / 16, mtiles - mg * (kWgRows / 16));
    return std::max(1, std::min(kWgMaxMT, (tiles + kWgWaves - 1) / kWgWaves));
}

int build_plan(Plan& P, const MpoCnnSpec* specs, int n, int B) {
    P.n = n;
    P.B = B;
    P.mem.resize(n);
    long long po = 0, ao = 0;
    auto palloc = [&](long long cnt) { long long o = po; po += (cnt + 63) / 64 * 64; return o; };
    auto aalloc = [&](long long cnt) { long long o = ao; ao += (cnt + 63) / 64 * 64; return o; };
    for (int i = 0; i < n; ++i) {
        const MpoCnnSpec& s = specs[i];
        Member& m = P.mem[i];
        if (s.nb_filters < 1 || s.nb_filters > 64 || s.kernel_size < 1 || s.kernel_size > 13 || s.pool_size < 1 ||
            s.dense < 1 || s.dense > 4096 || !(s.dropout >= 0.f && s.dropout < 1.f) || !(s.lr > 0.f)) {
            mpo::set_error("mpo_pop_create: member %d has unsupported spec (F=%d k=%d p=%d dense=%d lr=%g dropout=%g)", i,
                           s.nb_filters, s.kernel_size, s.pool_size, s.dense, s.lr, s.dropout);
            return MPO_ENOTSUP;
        }
        m.F = s.nb_filters; m.k = s.kernel_size; m.p = s.pool_size; m.dense = s.dense;
        m.H1 = kImg - m.k + 1;
        m.H2 = m.H1 - m.k + 1;
        if (m.H2 < 1) { mpo::set_error("mpo_pop_create: member %d kernel too large", i); return MPO_ENOTSUP; }
        m.s = m.H2 / m.p;
        if (m.s < 1) { mpo::set_error("mpo_pop_create: member %d pool larger than feature map", i); return MPO_ENOTSUP; }
        m.K1 = m.s * m.s * m.F;
        const int loss = s.options & MPO_LOSS_MASK, opt = s.options & MPO_OPT_MASK;
        if ((s.options & ~(MPO_LOSS_MASK | MPO_OPT_MASK)) || (loss != MPO_LOSS_BCE && loss != MPO_LOSS_CCE) ||
            (opt != MPO_OPT_ADAM && opt != MPO_OPT_SGD)) {
            mpo::set_error("mpo_pop_create: member %d has unsupported options 0x%x", i, (unsigned)s.options);
            return MPO_ENOTSUP;
        }
        m.loss = loss; m.opt = opt;
        m.lr = s.lr; m.rate = s.dropout; m.inv_keep = 1.f / (1.f - s.dropout); m.seed = s.seed;
        m.drop_thr = (unsigned)std::ceil((double)s.dropout * 16777216.0);
        m.nt = (m.F + 15) / 16;
        const int k = m.k, F = m.F, D = m.dense;
        m.w1 = palloc((long long)k * k * F); m.b1 = palloc(F);
        m.w2 = palloc((long long)k * k * F * F); m.b2 = palloc(F);
        m.w3 = palloc((long long)m.K1 * D); m.b3 = palloc(D);
        m.w4 = palloc((long long)D * kClasses); m.b4 = palloc(kClasses);
        m.pend = po;
        // wgrad sample groups (partial slabs reduced in a fixed order): 2 samples per
        // conv2 slab (r04: a 40-member population's conv2 weight gradient has too few
        // workgroups at 4: 6.75 -> 6.12 ms per step, 320 members unchanged 37.48 -> 37.39,
        // profiles/r04/train_probe_spg_i.log), 4 per conv1 slab (its GEMM is tiny).  A
        // function of the member only, never of the population: a member's trajectory
        // must not depend on who trains beside it (isolation tests, chunked populations)
        // r06: members whose conv2 weight gradient has >= wg_big m-groups of 512 rows (k^2 F + 1
        // rows) take wg_spg2_big = 4 samples per slab -- they launch g2 x m-groups workgroups, so
        // halving g2 still fills the chip and halves their slab writes / reduction: 37.10 -> 36.65
        // ms per 320-member step, 3.85 -> 3.82 at 40, 20 unchanged (profiles/r06/mnist/bc_*.log).
        // Still a function of the member alone (isolation); wg_spg2_big=0 restores one spg2
        const int mg2 = (k * k * F + 1 + kWgRows - 1) / kWgRows;
        const int big = plan_knob("wg_spg2_big", 4), bigmg = plan_knob("wg_big", 3);
        const int spg2 = std::max(1, big > 0 && mg2 >= bigmg ? big : plan_knob("wg_spg2", 2));
        const int spg1 = std::max(1, plan_knob("wg_spg1", 4));
        m.g2 = std::max(1, std::min(B, (B + spg2 - 1) / spg2));
        m.g1 = std::max(1, std::min(B, (B + spg1 - 1) / spg1));
        m.a1 = aalloc((long long)B * m.H1 * m.H1 * F);
        m.a2 = aalloc((long long)B * m.H2 * m.H2 * F);
        m.pd = aalloc((long long)B * m.K1);
        m.am = aalloc(((long long)B * m.K1 + 3) / 4);
        m.h = aalloc((long long)B * D);
        m.hd = aalloc((long long)B * D);
        m.z3 = aalloc((long long)B * kClasses);
        m.dz3 = aalloc((long long)B * kClasses);
        m.dh = aalloc((long long)B * D);
        m.dp = aalloc((long long)B * m.K1);
        m.dz2 = aalloc((long long)B * m.H2 * m.H2 * F);
        m.dz1 = aalloc((long long)B * m.H1 * m.H1 * F);
        m.w2t = aalloc((long long)(((k * k * ((F + 3) & ~3) + 15) & ~15) + kWSlack) * (m.nt * 16));
        m.w1p = aalloc((long long)(((k * k + 15) & ~15) + kWSlack) * (m.nt * 16));
        m.w2p = aalloc((long long)(((k * k * F + 15) & ~15) + kWSlack) * (m.nt * 16));
        m.wp1 = aalloc((long long)m.g1 * (k * k + 1) * F);
        m.wp2 = aalloc((long long)m.g2 * (k * k * F + 1) * F);
    }
    P.zero_off = aalloc(64);   // never written: the caller zero-initialises the arena
    P.n_params = po;
    P.act_floats = ao;

    // ---- work lists (LDS budgets per workgroup in KiB: A/B knobs, defaults tuned on MI355X)
    // r03: forward items of up to 256 pixels (4 m-tiles per wave) in <= 40 KiB (4 workgroups per CU) where
    // rows in [rmax/2, rmax] fit, else <= 100 KiB: conv2 fwd 9.66 -> 8.53 ms per 320-member batch
    // (profiles/r03/train_sweep_mt4_budget_am.log; 128-pixel items at 52/78 KiB were r01-r02's plan)
    // r06, after dgfwd + wgpair (profiles/r06/mnist/av_*, aw_*): a 30 KiB first budget, 37.41 / 37.28 ->
    // 37.13 / 37.08 ms per 320-member step, 3.95 -> 3.86 ms at 40, 1.633 -> 1.642 at 20 (24 and 36 alike)
    const int kc1 = plan_knob("conv_kb1", 30), kc2 = plan_knob("conv_kb2", 100);
    const int kdg = plan_knob("dg_kb", 78);
    std::vector<size_t> L1(n), L2(n), LD(n), LDF(n), LW1(n), LW2(n);   // per-member LDS bytes per op
    for (int i = 0; i < n; ++i) {
        const Member& m = P.mem[i];
        const int k = m.k, F = m.F, nt = m.nt;
        if (i == 0) P.conv_mt = plan_knob("conv_mt", 4) == 2 ? 2 : 4;
        if (i == 0) P.side.enabled = plan_knob("streams", 3) >= 2;
        if (i == 0) P.side2.enabled = plan_knob("streams", 3) >= 3;
        if (i == 0) P.side2.slot = 1;
        if (i == 0) P.side3.enabled = P.side.enabled && plan_knob("wgs", 2) >= 2;
        if (i == 0) P.side3.slot = 2;
        if (i == 0) P.side4.enabled = P.side2.enabled && plan_knob("dgs", 3) >= 3;
        if (i == 0) P.side4.slot = 3;
        const int mcap = P.conv_mt * 64;   // 4 waves x conv_mt m-tiles of 16 pixels
        const int R1 = choose_rows(m.H1, [&](int R) { return conv_lds_bytes(R + k - 1, kImg, 1, m.H1, k * k, nt); }, kc1, kc2, mcap);
        const int R2 = choose_rows(m.H2, [&](int R) { return conv_lds_bytes(R + k - 1, m.H1, F, m.H2, k * k * F, nt); }, kc1, kc2, mcap);
        // dgrad: 4x4-pixel tiles in bands of 4 rows, <= 16 tiles (4 per wave) per chunk:
        // R = 4 * floor(16 / CT); 4-row bands fewer if the LDS budget asks for it
        const size_t dgb = (size_t)kdg << 10;
        // r03: at most 12 tiles (3 per wave): conv2 dgrad 15.40 -> 15.15 ms per 320-member batch
        // (profiles/r03/train_sweep_dgtiles_ap.log; 16 was r01-r02's, 8 measured 16.96)
        if (i == 0) P.dg_tiles = std::max(1, std::min(16, plan_knob("dg_tiles", 12)));
        int Rd = 4 * std::max(1, P.dg_tiles / ((m.H1 + 3) / 4));
        while (Rd > 4 && dgrad_lds_bytes(Rd, k, F, m.H2) > dgb) Rd -= 4;
        const size_t l1 = conv_lds_bytes(R1 + k - 1, kImg, 1, m.H1, k * k, nt);
        const size_t l2 = conv_lds_bytes(R2 + k - 1, m.H1, F, m.H2, k * k * F, nt);
        size_t ld = dgrad_lds_bytes(Rd, k, F, m.H2);
        // the zero-bordered forward formulation (k small: (H1 / H2)^2 of padded work)
        // r06, MI355X, 320 members (profiles/r06/mnist/ao_*, ap_*): k <= 4 -> 36.70 ms per train step
        // 35.85 (k = 4 carries it; k = 2-3 neutral), with an 80 KiB first LDS budget 35.67; adding k =
        // 5..10 one at a time: 5-7 within noise, 8 +0.2, 9 +0.6, 10 +2.2 ms.  Bits unchanged.
        if (i == 0) P.dgfwd = plan_knob("dgfwd", 4);
        if (i == 0) P.dgfset = plan_knob("dgfset", 0);
        const bool fwd_dg = k <= P.dgfwd || ((P.dgfset >> k) & 1);
        const int F4 = (F + 3) & ~3, Hp = m.H1 + k - 1;
        const int Rf = choose_rows(m.H1, [&](int R) { return conv_lds_bytes(R + k - 1, Hp, F4, m.H1, k * k * F4, nt); },
                                   plan_knob("dgf_kb1", 80), plan_knob("dgf_kb2", kc2), mcap);
        if (fwd_dg) ld = conv_lds_bytes(Rf + k - 1, Hp, F4, m.H1, k * k * F4, nt);
        L1[i] = l1; L2[i] = l2; LD[i] = ld; LDF[i] = ld;
        for (int b = 0; b < B; ++b) {
            for (int y = 0; y < m.H1; y += R1) P.conv1.push_back({i, b, y, std::min(R1, m.H1 - y)});
            for (int y = 0; y < m.H2; y += R2) P.conv2.push_back({i, b, y, std::min(R2, m.H2 - y)});
            if (fwd_dg)
                for (int y = 0; y < m.H1; y += Rf) P.dgf.push_back({i, b, y, std::min(Rf, m.H1 - y)});
            else
                for (int y = 0; y < m.H1; y += Rd) P.dgrad.push_back({i, b, y, std::min(Rd, m.H1 - y)});
            P.per_sample.push_back({i, b});
        }
        P.lds_conv_max = std::max({P.lds_conv_max, l1, l2, ld});
        // wgrad items: (member, 512-row m-group, sample group)
        if (i == 0) P.wgrpb = plan_knob("wgrpb", 2) == 1 ? 1 : 2;
        // r06, MI355X (profiles/r06/mnist/as_*.log): 37.70 -> 37.29 ms per 320-member step,
        // 1.64 -> 1.63 ms at 20; losses bit-identical (a padding pixel's MFMA product is an exact zero)
        if (i == 0) P.wgpair = plan_knob("wgpair", 1);
        const size_t lw2 = wg_lds_bytes(k, m.H1, F, m.H2, F, P.wgrpb);
        const size_t lw1 = wg_lds_bytes(k, kImg, 1, m.H1, F);
        LW2[i] = lw2; LW1[i] = lw1;
        const int K2 = k * k * F, K1w = k * k;
        for (int g = 0; g < m.g2; ++g) {
            const int b0 = (int)((long long)B * g / m.g2), b1 = (int)((long long)B * (g + 1) / m.g2);
            for (int mg = 0; mg * kWgRows <= K2; ++mg) P.wg2.push_back({i, mg, b0, b1, g, wg_mt(K2, mg)});
        }
        // conv1_wgrad_kernel: every m-tile in one wave, MT bucketed to 1, 2, 4 or 7
        const int t1 = (K1w + 1 + 15) / 16, mt1 = t1 <= 1 ? 1 : t1 <= 2 ? 2 : t1 <= 4 ? 4 : 7;
        LW1[i] = (size_t)w1_lds_floats((B + m.g1 - 1) / m.g1, mt1, nt) * sizeof(float);
        for (int g = 0; g < m.g1; ++g) {
            const int b0 = (int)((long long)B * g / m.g1), b1 = (int)((long long)B * (g + 1) / m.g1);
            P.wg1.push_back({i, 0, b0, b1, g, mt1});
        }
        P.lds_wg_max = std::max({P.lds_wg_max, lw2, lw1});
        auto tiles = [&](std::vector<GemmItem>& v, int M, int N) {
            for (int m0 = 0; m0 < M; m0 += 64)
                for (int n0 = 0; n0 < N; n0 += 64) v.push_back({i, m0, n0, 0});
        };
        tiles(P.d1f, B, m.dense);
        tiles(P.d2f, B, kClasses);
        tiles(P.d2w, m.dense, kClasses);
        tiles(P.d2d, B, m.dense);
        tiles(P.d1w, m.K1, m.dense);
        tiles(P.d1d, B, m.K1);
        P.per_member.push_back({i, 0});
        for (int c = 2; c < 4; ++c) P.colsum.push_back({i, c});
        P.wred.push_back({i, 1});   // conv2 slabs: items [0, n) (reduced on the side stream)
        const long long np_ = m.pend - m.w1;
        for (long long c = 0; c * P.adam_chunk < np_; ++c) P.adam.push_back({i, (int)c});
    }
    if (P.lds_conv_max > 160 * 1024 || P.lds_wg_max > 160 * 1024) {
        mpo::set_error("mpo_pop_create: LDS plan exceeds 160 KiB (conv %zu, wgrad %zu)", P.lds_conv_max, P.lds_wg_max);
        return MPO_ENOTSUP;
    }
    for (int i = 0; i < n; ++i) P.wred.push_back({i, 0});   // conv1 slabs: items [n, 2n)
    long long wmax = 0;
    for (auto& m : P.mem) wmax = std::max(wmax, (long long)m.k * m.k * m.F * m.F + m.F);
    P.wred_blocks = (int)((wmax + P.wred_per_block - 1) / P.wred_per_block);
    // Small populations (a distributed shard, configs[0]) launch too few workgroups per occupancy class
    // to fill the chip.  Merging every class of an (NT, sub) bucket (mode 1) measured on MI355X
    // (profiles/r05/occmerge_o.log): 20 members 3.82 -> 3.52 ms, 40: 5.93 -> 5.70, 80: 10.94 -> 10.96,
    // 160: 19.81 -> 20.30, 320: 36.92 -> 39.06 ms per train step.  Merging only adjacent classes
    // short of one full wave (mode 2, the default): 20: 3.53, 40: 5.56-5.59, 80: 10.63-10.67,
    // 320: 36.81-36.95 (separate classes 36.87) -- profiles/r05/occmerge2_*.log.  The segmenting
    // changes no arithmetic.
    const int occ = plan_knob("occmerge", 2);
    bucket_segs(P.conv1, P.bc1, P.mem, L1, occ);
    bucket_segs(P.conv2, P.bc2, P.mem, L2, occ);
    bucket_segs(P.dgrad, P.bdg, P.mem, LD, occ);
    bucket_segs(P.dgf, P.bdf, P.mem, LDF, occ);
    bucket_segs(P.wg1, P.bw1, P.mem, LW1, occ);
    bucket_segs(P.wg2, P.bw2, P.mem, LW2, occ);
    const int xc = plan_knob("xcd", 4);
    xcd_deal(P.conv1, P.bc1, xc);
    xcd_deal(P.conv2, P.bc2, xc);
    xcd_deal(P.dgrad, P.bdg, xc);
    xcd_deal(P.dgf, P.bdf, xc);
    xcd_deal(P.wg1, P.bw1, xc);
    xcd_deal(P.wg2, P.bw2, xc);

    // ---- serialise tables (one device upload)
    size_t off = 0;
    auto put = [&](const void* src, size_t bytes) {
        off = mpo::align_up(off, 256);
        const size_t o = off;
        P.host_tables.resize(off + bytes);
        if (bytes) std::copy_n(static_cast<const char*>(src), bytes, P.host_tables.data() + o);
        off += bytes;
        return o;
    };
    P.off_mem = put(P.mem.data(), P.mem.size() * sizeof(Member));
    P.off_conv1 = put(P.conv1.data(), P.conv1.size() * sizeof(ConvItem));
    P.off_conv2 = put(P.conv2.data(), P.conv2.size() * sizeof(ConvItem));
    P.off_dgrad = put(P.dgrad.data(), P.dgrad.size() * sizeof(ConvItem));
    P.off_dgf = put(P.dgf.data(), P.dgf.size() * sizeof(ConvItem));
    P.off_wg1 = put(P.wg1.data(), P.wg1.size() * sizeof(WgItem));
    P.off_wg2 = put(P.wg2.data(), P.wg2.size() * sizeof(WgItem));
    P.off_d1f = put(P.d1f.data(), P.d1f.size() * sizeof(GemmItem));
    P.off_d2f = put(P.d2f.data(), P.d2f.size() * sizeof(GemmItem));
    P.off_d2w = put(P.d2w.data(), P.d2w.size() * sizeof(GemmItem));
    P.off_d2d = put(P.d2d.data(), P.d2d.size() * sizeof(GemmItem));
    P.off_d1w = put(P.d1w.data(), P.d1w.size() * sizeof(GemmItem));
    P.off_d1d = put(P.d1d.data(), P.d1d.size() * sizeof(GemmItem));
    P.off_pm = put(P.per_member.data(), P.per_member.size() * sizeof(MItem));
    P.off_ps = put(P.per_sample.data(), P.per_sample.size() * sizeof(MItem));
    P.off_cs = put(P.colsum.data(), P.colsum.size() * sizeof(MItem));
    P.off_wr = put(P.wred.data(), P.wred.size() * sizeof(MItem));
    P.off_adam = put(P.adam.data(), P.adam.size() * sizeof(MItem));
    P.table_bytes = mpo::align_up(off, 256);
    P.host_tables.resize(P.table_bytes);
    return MPO_OK;
}

template <class T>
const T* dev_table(const Plan& P, size_t off) {
    return reinterpret_cast<const T*>(P.table_base + off);
}

template <int OP, int NT>
hipError_t launch_conv_nt(const StepArgs& a, const ConvItem* items, int count, size_t lds, hipStream_t s) {
    if (count <= 0) return hipSuccess;
    auto kern = a.conv_mt == 4 ? conv_img_kernel<OP, NT, 4> : conv_img_kernel<OP, NT, 2>;
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(kern, dim3(count), dim3(256), lds, s, a, items);
    return hipGetLastError();
}

template <int NT>
hipError_t launch_dgrad_nt(const StepArgs& a, const ConvItem* items, int count, size_t lds, hipStream_t s) {
    if (count <= 0) return hipSuccess;
    auto kern = conv_dgrad_kernel<NT>;
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(kern, dim3(count), dim3(256), lds, s, a, items);
    return hipGetLastError();
}

template <int OP, int NT, int RPB>
auto wg_kernel(int mt) {
    return mt == 1 ? conv_wgrad_kernel<OP, NT, 1, RPB> : mt == 2 ? conv_wgrad_kernel<OP, NT, 2, RPB>
         : mt == 3 ? conv_wgrad_kernel<OP, NT, 3, RPB> : conv_wgrad_kernel<OP, NT, 4, RPB>;
}

template <int OP, int NT>
hipError_t launch_wg_nt(const StepArgs& a, const WgItem* items, int count, size_t lds, int mt, hipStream_t s) {
    if (count <= 0) return hipSuccess;
    auto kern = a.wgrpb == 2 ? wg_kernel<OP, NT, 2>(mt) : wg_kernel<OP, NT, 1>(mt);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(kern, dim3(count), dim3(kWgThreads), lds, s, a, items);
    return hipGetLastError();
}

template <int NT>
hipError_t launch_wg1_wave_nt(const StepArgs& a, const WgItem* items, int count, size_t lds, int mt, hipStream_t s) {
    if (count <= 0) return hipSuccess;
    auto kern = mt == 1 ? conv1_wgrad_kernel<NT, 1> : mt == 2 ? conv1_wgrad_kernel<NT, 2>
              : mt == 4 ? conv1_wgrad_kernel<NT, 4> : conv1_wgrad_kernel<NT, 7>;
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(kern, dim3(count), dim3(kW1Waves * 64), lds, s, a, items);
    return hipGetLastError();
}

// s2 (optional): segments alternate between s and s2 (independent launches)
template <class Fn>
hipError_t launch_segs(Plan& P, const Bucketed& bk, const char* name, hipStream_t s, Fn launch_nt,
                       hipStream_t s2 = nullptr, hipStream_t s3 = nullptr) {
    // segments dealt round-robin over s, s2 (, s3)
    const hipStream_t st[3] = {s, s2, s3};
    const int ns = s2 ? (s3 ? 3 : 2) : 1;
    int i = 0;
    for (const Seg& sg : bk.segs) {
        if (hipError_t e = launch_nt(sg, st[i++ % ns])) return e;
        P.timer.mark(std::string(name) + "/nt" + std::to_string(sg.nt) + (sg.sub ? "/mt" + std::to_string(sg.sub) : "") +
                         (P.timer_detail ? "/occ" + std::to_string(lds_class(sg.lds)) + "/n" + std::to_string(sg.end - sg.begin) : ""),
                     s);
    }
    return hipSuccess;
}

#define MPO_NT_SWITCH(FN, sg, ...)                                     \
    ((sg).nt == 1 ? FN<1>(__VA_ARGS__)                                 \
     : (sg).nt == 2 ? FN<2>(__VA_ARGS__)                               \
     : (sg).nt == 3 ? FN<3>(__VA_ARGS__) : FN<4>(__VA_ARGS__))

template <int OP>
struct ConvLaunch {
    template <int NT>
    static hipError_t go(const StepArgs& a, const ConvItem* items, int count, size_t lds, hipStream_t s) {
        return launch_conv_nt<OP, NT>(a, items, count, lds, s);
    }
};

template <int OP>
hipError_t launch_conv(Plan& P, const StepArgs& a, size_t table_off, const Bucketed& bk, hipStream_t s,
                       hipStream_t s2 = nullptr) {
    const ConvItem* base = dev_table<ConvItem>(P, table_off);
    return launch_segs(P, bk, OP == CONV1_FWD ? "conv1_fwd" : "conv2_fwd", s, [&](const Seg& sg, hipStream_t st) {
        return MPO_NT_SWITCH(ConvLaunch<OP>::template go, sg, a, base + sg.begin, sg.end - sg.begin, sg.lds, st);
    }, s2);
}

hipError_t launch_dgrad(Plan& P, const StepArgs& a, hipStream_t s, hipStream_t s2 = nullptr, hipStream_t s3 = nullptr) {
    const ConvItem* base = dev_table<ConvItem>(P, P.off_dgrad);
    const ConvItem* fbase = dev_table<ConvItem>(P, P.off_dgf);
    if (hipError_t e = launch_segs(P, P.bdf, "conv2_dgrad_fwd", s, [&](const Seg& sg, hipStream_t st) {
            return MPO_NT_SWITCH(ConvLaunch<CONV2_DGRAD>::template go, sg, a, fbase + sg.begin, sg.end - sg.begin, sg.lds, st);
        }, s2, s3))
        return e;
    return launch_segs(P, P.bdg, "conv2_dgrad", s, [&](const Seg& sg, hipStream_t st) {
        return MPO_NT_SWITCH(launch_dgrad_nt, sg, a, base + sg.begin, sg.end - sg.begin, sg.lds, st);
    }, s2, s3);
}

template <int OP>
struct WgLaunch {
    template <int NT>
    static hipError_t go(const StepArgs& a, const WgItem* items, int count, size_t lds, int mt, hipStream_t s) {
        return launch_wg_nt<OP, NT>(a, items, count, lds, mt, s);
    }
};

template <int OP>
hipError_t launch_wg(Plan& P, const StepArgs& a, size_t table_off, const Bucketed& bk, hipStream_t s,
                     hipStream_t s_alt = nullptr) {
    const WgItem* base = dev_table<WgItem>(P, table_off);
    return launch_segs(P, bk, OP == WG_CONV1 ? "conv1_wgrad" : "conv2_wgrad", s, [&](const Seg& sg, hipStream_t st) {
        if constexpr (OP == WG_CONV1)
            return MPO_NT_SWITCH(launch_wg1_wave_nt, sg, a, base + sg.begin, sg.end - sg.begin, sg.lds, sg.sub, st);
        else
            return MPO_NT_SWITCH(WgLaunch<OP>::template go, sg, a, base + sg.begin, sg.end - sg.begin, sg.lds, sg.sub, st);
    }, s_alt);
}

template <int OP>
hipError_t launch_dense(const Plan& P, const StepArgs& a, size_t off, size_t count, hipStream_t s) {
    if (!count) return hipSuccess;
    hipLaunchKernelGGL(dense_kernel<OP>, dim3((unsigned)count), dim3(256), 0, s, a, dev_table<GemmItem>(P, off));
    return hipGetLastError();
}

StepArgs make_args(const Plan& P, const float* x, const int* labels, const int* order, long long order_stride,
                   long long row0, int step, int train) {
    StepArgs a;
    a.mem = dev_table<Member>(P, P.off_mem);
    a.params = P.params;
    a.grads = P.grads;
    a.act = P.act;
    a.x = x;
    a.labels = labels;
    a.order = order;
    a.order_stride = order_stride;
    a.row0 = row0;
    a.B = P.B;
    a.step = step;
    a.train = train;
    a.loss_out = nullptr;
    a.loss_sum = nullptr;
    a.correct = nullptr;
    a.debug = P.debug;
    a.conv_mt = P.conv_mt;
    a.wgrpb = P.wgrpb;
    a.wgpair = P.wgpair;
    a.zero_off = P.zero_off;
    return a;
}

int forward(Plan& P, const StepArgs& a, hipStream_t s) {
    P.timer.mark("start", s);
    // padded / rotated weight copies for this step's convolutions
    hipLaunchKernelGGL(flip_w2_kernel, dim3(64, (unsigned)P.n), dim3(256), 0, s, a, dev_table<MItem>(P, P.off_pm));
    MPO_LAUNCH_CHECK();
    P.timer.mark("flip_w2", s);
    MPO_HIP(launch_conv<CONV1_FWD>(P, a, P.off_conv1, P.bc1, s));
    if (hipStream_t s2 = P.timer.on ? nullptr : P.side.get(s)) {   // profiled steps stay serial
        MPO_HIP(P.side.fork(s, s2));
        MPO_HIP(launch_conv<CONV2_FWD>(P, a, P.off_conv2, P.bc2, s, s2));
        MPO_HIP(P.side.join(s, s2));
    } else {
        MPO_HIP(launch_conv<CONV2_FWD>(P, a, P.off_conv2, P.bc2, s));
    }
    hipLaunchKernelGGL(pool_fwd_kernel, dim3((unsigned)P.per_sample.size()), dim3(256), 0, s, a,
                       dev_table<MItem>(P, P.off_ps));
    MPO_LAUNCH_CHECK();
    P.timer.mark("pool_fwd", s);
    MPO_HIP(launch_dense<D1_FWD>(P, a, P.off_d1f, P.d1f.size(), s));
    MPO_HIP(launch_dense<D2_FWD>(P, a, P.off_d2f, P.d2f.size(), s));
    P.timer.mark("dense_fwd", s);
    hipLaunchKernelGGL(softmax_bce_kernel, dim3((unsigned)P.n), dim3(256), 0, s, a, dev_table<MItem>(P, P.off_pm));
    MPO_LAUNCH_CHECK();
    P.timer.mark("softmax_bce", s);
    return MPO_OK;
}

}  // namespace

// ===========================================================================
extern "C" {

int mpo_pop_create(const MpoCnnSpec* specs, int n_members, int batch, void** handle) {
    MPO_GUARD_BEGIN
    MPO_CHECK_ARG(specs && handle, "mpo_pop_create: null pointer");
    MPO_CHECK_ARG(n_members > 0 && batch > 0 && batch <= 256, "mpo_pop_create: n_members=%d batch=%d (1..256)",
                  n_members, batch);
    auto P = std::make_unique<Plan>();
    P->timer.on = env_int("MPO_POP_PROFILE", 0) != 0;
    P->debug = plan_knob("dbg", env_int("MPO_POP_DEBUG", 0));
    P->timer_detail = env_int("MPO_POP_PROFILE", 0) > 1;
    int rc = build_plan(*P, specs, n_members, batch);
    if (rc) return rc;
    *handle = P.release();
    return MPO_OK;
    MPO_GUARD_END
}

int mpo_pop_destroy(void* handle) {
    delete static_cast<Plan*>(handle);
    return MPO_OK;
}

int mpo_pop_sizes(const void* handle, MpoPopSizes* out) {
    MPO_CHECK_ARG(handle && out, "mpo_pop_sizes: null pointer");
    const Plan& P = *static_cast<const Plan*>(handle);
    out->n_params = P.n_params;
    out->act_floats = P.act_floats;
    out->table_bytes = (int64_t)P.table_bytes;
    out->n_members = P.n;
    out->batch = P.B;
    return MPO_OK;
}

int mpo_pop_param_layout(const void* handle, int member, int64_t* offsets) {
    MPO_CHECK_ARG(handle && offsets, "mpo_pop_param_layout: null pointer");
    const Plan& P = *static_cast<const Plan*>(handle);
    MPO_CHECK_ARG(member >= 0 && member < P.n, "mpo_pop_param_layout: member %d out of range", member);
    const Member& m = P.mem[member];
    const long long o[9] = {m.w1, m.b1, m.w2, m.b2, m.w3, m.b3, m.w4, m.b4, m.pend};
    for (int i = 0; i < 9; ++i) offsets[i] = o[i];
    return MPO_OK;
}

int mpo_pop_act_layout(const void* handle, int member, int64_t* offsets) {
    MPO_CHECK_ARG(handle && offsets, "mpo_pop_act_layout: null pointer");
    const Plan& P = *static_cast<const Plan*>(handle);
    MPO_CHECK_ARG(member >= 0 && member < P.n, "mpo_pop_act_layout: member %d out of range", member);
    const Member& m = P.mem[member];
    const long long o[15] = {m.a1, m.a2, m.pd, m.am, m.h, m.hd, m.z3, m.dz3, m.dh, m.dp, m.dz2, m.dz1, m.w2t, m.wp1, m.wp2};
    for (int i = 0; i < 15; ++i) offsets[i] = o[i];
    return MPO_OK;
}

int mpo_pop_bind(void* handle, float* params, float* grads, float* adam_m, float* adam_v, float* act, void* tables,
                 void* stream) {
    MPO_GUARD_BEGIN
    MPO_CHECK_ARG(handle && params && grads && adam_m && adam_v && act && tables, "mpo_pop_bind: null pointer");
    Plan& P = *static_cast<Plan*>(handle);
    P.params = params;
    P.grads = grads;
    P.m = adam_m;
    P.v = adam_v;
    P.act = act;
    P.table_base = static_cast<char*>(tables);
    MPO_HIP(hipMemcpyAsync(tables, P.host_tables.data(), P.table_bytes, hipMemcpyHostToDevice,
                           static_cast<hipStream_t>(stream)));
    P.bound = true;
    return MPO_OK;
    MPO_GUARD_END
}

int mpo_pop_train_step(void* handle, const float* x, const int32_t* labels, const int32_t* order, int64_t order_stride,
                       int64_t row0, int32_t step, float* loss_out, void* stream) {
    MPO_GUARD_BEGIN
    MPO_CHECK_ARG(handle && x && labels && order && loss_out, "mpo_pop_train_step: null pointer");
    Plan& P = *static_cast<Plan*>(handle);
    MPO_CHECK_ARG(P.bound, "mpo_pop_train_step: call mpo_pop_bind first");
    MPO_CHECK_ARG(step >= 0, "mpo_pop_train_step: step must be >= 0");
    hipStream_t s = static_cast<hipStream_t>(stream);
    StepArgs a = make_args(P, x, labels, order, order_stride, row0, step, 1);
    a.loss_out = loss_out;
    int rc = forward(P, a, s);
    if (rc) return rc;
    // backward.  With the side stream s2: each weight gradient runs on s2 beside the
    // input gradient that follows it on s (disjoint outputs; s2 stays one stream, so
    // its work keeps its own order), the conv2 slab reduction right after the conv2
    // weight gradient, and s joins s2 before Adam.
    hipStream_t s2 = P.timer.on ? nullptr : P.side.get(s);
    const MItem* wred = dev_table<MItem>(P, P.off_wr);
    const unsigned nm = (unsigned)P.n;
    if (s2) {
        MPO_HIP(P.side.fork(s, s2));                                        // dz3 ready
        MPO_HIP(launch_dense<D2_WGRAD>(P, a, P.off_d2w, P.d2w.size(), s2));
        MPO_HIP(launch_dense<D2_DGRAD>(P, a, P.off_d2d, P.d2d.size(), s));
        MPO_HIP(P.side.fork(s, s2));                                        // dh ready
        MPO_HIP(launch_dense<D1_WGRAD>(P, a, P.off_d1w, P.d1w.size(), s2));
        MPO_HIP(launch_dense<D1_DGRAD>(P, a, P.off_d1d, P.d1d.size(), s));
    } else {
        MPO_HIP(launch_dense<D2_WGRAD>(P, a, P.off_d2w, P.d2w.size(), s));
        MPO_HIP(launch_dense<D2_DGRAD>(P, a, P.off_d2d, P.d2d.size(), s));
        MPO_HIP(launch_dense<D1_WGRAD>(P, a, P.off_d1w, P.d1w.size(), s));
        MPO_HIP(launch_dense<D1_DGRAD>(P, a, P.off_d1d, P.d1d.size(), s));
    }
    P.timer.mark("dense_bwd", s);
    hipLaunchKernelGGL(pool_bwd_kernel, dim3((unsigned)P.per_sample.size()), dim3(256), 0, s, a,
                       dev_table<MItem>(P, P.off_ps));
    MPO_LAUNCH_CHECK();
    P.timer.mark("pool_bwd", s);
    if (s2) {
        // conv2 weight gradient (a1, dz2 -> slabs -> dw2) beside the input gradient and
        // the conv1 weight gradient (dz2 -> dz1 -> slabs -> dw1): disjoint outputs
        MPO_HIP(P.side.fork(s, s2));                                        // dz2 ready
        hipStream_t s4 = P.side3.get(s);   // disjoint slab rows per bucket: alternating buckets may overlap
        if (s4) MPO_HIP(P.side3.fork(s, s4));
        MPO_HIP(launch_wg<WG_CONV2>(P, a, P.off_wg2, P.bw2, s2, s4));
        if (s4) MPO_HIP(P.side3.join(s2, s4));                              // the slab reduction reads all of them
        hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)P.wred_blocks, nm), dim3(256), 0, s2, a, wred,
                           P.wred_per_block);
        MPO_LAUNCH_CHECK();
        if (hipStream_t s3 = P.side2.get(s)) {   // input-gradient buckets over s and s3 (disjoint rows of dz1)
            MPO_HIP(P.side2.fork(s, s3));
            hipStream_t s5 = P.side4.get(s);
            if (s5) MPO_HIP(P.side4.fork(s, s5));
            MPO_HIP(launch_dgrad(P, a, s, s3, s5));
            MPO_HIP(P.side2.join(s, s3));
            if (s5) MPO_HIP(P.side4.join(s, s5));
        } else {
            MPO_HIP(launch_dgrad(P, a, s));
        }
        MPO_HIP(launch_wg<WG_CONV1>(P, a, P.off_wg1, P.bw1, s));
        hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)P.wred_blocks, nm), dim3(256), 0, s, a, wred + nm,
                           P.wred_per_block);
        MPO_LAUNCH_CHECK();
        MPO_HIP(P.side.join(s, s2));
    } else {
        MPO_HIP(launch_dgrad(P, a, s));
        MPO_HIP(launch_wg<WG_CONV2>(P, a, P.off_wg2, P.bw2, s));
        MPO_HIP(launch_wg<WG_CONV1>(P, a, P.off_wg1, P.bw1, s));
        hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)P.wred_blocks, 2 * nm), dim3(256), 0, s, a, wred,
                           P.wred_per_block);
        MPO_LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(colsum_kernel, dim3((unsigned)P.colsum.size()), dim3(256), 0, s, a, dev_table<MItem>(P, P.off_cs));
    MPO_LAUNCH_CHECK();
    P.timer.mark("wgrad_reduce", s);
    hipLaunchKernelGGL(adam_kernel, dim3((unsigned)P.adam.size()), dim3(256), 0, s, a, dev_table<MItem>(P, P.off_adam),
                       P.params, P.m, P.v, step + 1, 0.9f, 0.999f, 1e-8f, P.adam_chunk);
    MPO_LAUNCH_CHECK();
    P.timer.mark("adam", s);
    P.timer.finish();
    return MPO_OK;
    MPO_GUARD_END
}

int mpo_pop_eval_step(void* handle, const float* x, const int32_t* labels, const int32_t* order, int64_t order_stride,
                      int64_t row0, float* loss_sum, int32_t* correct, void* stream) {
    MPO_GUARD_BEGIN
    MPO_CHECK_ARG(handle && x && labels && order && loss_sum && correct, "mpo_pop_eval_step: null pointer");
    Plan& P = *static_cast<Plan*>(handle);
    MPO_CHECK_ARG(P.bound, "mpo_pop_eval_step: call mpo_pop_bind first");
    StepArgs a = make_args(P, x, labels, order, order_stride, row0, 0, 0);
    a.loss_sum = loss_sum;
    a.correct = correct;
    const int rc = forward(P, a, static_cast<hipStream_t>(stream));
    P.timer.finish();
    return rc;
    MPO_GUARD_END
}

int mpo_pop_profile(void* handle, char* buf, size_t cap, int reset) {
    MPO_CHECK_ARG(handle && (buf || !cap), "mpo_pop_profile: null pointer");
    Plan& P = *static_cast<Plan*>(handle);
    std::string out;
    for (const auto& pr : P.timer.acc) {
        char line[128];
        snprintf(line, sizeof(line), "%s %.6f\n", pr.first.c_str(), pr.second);
        out += line;
    }
    if (cap) {
        const size_t n = std::min(cap - 1, out.size());
        std::copy_n(out.data(), n, buf);
        buf[n] = 0;
    }
    if (reset) P.timer.acc.clear();
    return P.timer.on ? MPO_OK : MPO_ENOTSUP;
}

int mpo_kfold_gather(const float* X, const int32_t* idx, int64_t rows, int row_elems, float* out, void* stream) {
    MPO_GUARD_BEGIN
    MPO_CHECK_ARG(X && idx && out, "mpo_kfold_gather: null pointer");
    MPO_CHECK_ARG(rows >= 0 && row_elems > 0, "mpo_kfold_gather: bad shape");
    if (rows == 0) return MPO_OK;
    const unsigned gy = (unsigned)std::min<int64_t>(rows, 65535);
    const unsigned gz = (unsigned)((rows + 65534) / 65535);
    const unsigned gx = (unsigned)std::min(8, (row_elems + 255) / 256);
    hipLaunchKernelGGL(kfold_gather_kernel, dim3(gx, gy, gz), dim3(256), 0, static_cast<hipStream_t>(stream), X, idx,
                       (long long)rows, row_elems, out);
    MPO_LAUNCH_CHECK();
    return MPO_OK;
    MPO_GUARD_END
}

}  // extern "C"
