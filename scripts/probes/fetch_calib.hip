// Calibration of rocprofv3 FETCH_SIZE / WRITE_SIZE for the access widths the
// training and DenseNet kernels use (diagnostic, not part of the library).
// MI355X_MICROARCH.md calibrates FETCH_SIZE only for 16 B/lane streaming reads
// (it reports half the bytes) and WRITE_SIZE for 16 B/lane stores; cnn.hip reads
// with 4 B/lane loads (dword activations and weight fragments, LDS-DMA dwords).
// Each kernel below moves exactly 1 GiB (4x the 256 MiB Infinity Cache) once:
//   rd_dword   contiguous 4 B/lane loads (stage_row, the activation staging)
//   rd_dwordx2 contiguous 8 B/lane loads (fp64 rows)
//   rd_dwordx4 contiguous 16 B/lane loads (the guide's calibrated case)
//   rd_frag    4 B/lane, 16 lanes per 64 B segment, 4 segments 256 B apart per
//              instruction (the conv weight-fragment pattern of cnn.hip)
//   rd_ldsdma  global_load_lds_dword, 4 B/lane (conv_wgrad's row DMA)
//   wr_dword / wr_dwordx4 / wr_frag: the same patterns as stores
// usage: rocprofv3 --pmc FETCH_SIZE -- ./fetch_calib   (then WRITE_SIZE)
#include <hip/hip_runtime.h>

#include <cstdio>

namespace {

constexpr size_t kFloats = size_t(1) << 28;   // 1 GiB
constexpr int kThreads = 256;
constexpr int kBlocks = 256 * 16;

typedef __attribute__((address_space(3))) void* lds_ptr_t;

__global__ __launch_bounds__(kThreads) void rd_dword(const float* __restrict__ s, float* out) {
    float acc = 0.f;
    const size_t stride = size_t(gridDim.x) * kThreads;
    for (size_t i = size_t(blockIdx.x) * kThreads + threadIdx.x; i < kFloats; i += stride) acc += s[i];
    if (acc == 12345.f) out[threadIdx.x] = acc;   // keeps the loads; never taken on zero data
}

__global__ __launch_bounds__(kThreads) void rd_dwordx2(const double* __restrict__ s, float* out) {
    double acc = 0.0;
    const size_t stride = size_t(gridDim.x) * kThreads;
    for (size_t i = size_t(blockIdx.x) * kThreads + threadIdx.x; i < kFloats / 2; i += stride) acc += s[i];
    if (acc == 12345.0) out[threadIdx.x] = (float)acc;
}

__global__ __launch_bounds__(kThreads) void rd_dwordx4(const float4* __restrict__ s, float* out) {
    float acc = 0.f;
    const size_t stride = size_t(gridDim.x) * kThreads;
    for (size_t i = size_t(blockIdx.x) * kThreads + threadIdx.x; i < kFloats / 4; i += stride) {
        const float4 v = s[i];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 12345.f) out[threadIdx.x] = acc;
}

// one wave covers a 256-float block per 4 instructions: lane (krow, kcol) reads
// block[krow * 64 + j * 16 + kcol], j = 0..3
__global__ __launch_bounds__(kThreads) void rd_frag(const float* __restrict__ s, float* out) {
    float acc = 0.f;
    const int lane = threadIdx.x & 63, krow = lane >> 4, kcol = lane & 15;
    const size_t wave = (size_t(blockIdx.x) * kThreads + threadIdx.x) >> 6;
    const size_t nwaves = (size_t(gridDim.x) * kThreads) >> 6;
    for (size_t b = wave; b < kFloats / 256; b += nwaves) {
        const float* p = s + b * 256 + krow * 64 + kcol;
#pragma unroll
        for (int j = 0; j < 4; ++j) acc += p[j * 16];
    }
    if (acc == 12345.f) out[threadIdx.x] = acc;
}

__global__ __launch_bounds__(kThreads) void rd_ldsdma(const float* __restrict__ s, float* out) {
    __shared__ float buf[kThreads];
    float acc = 0.f;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const size_t wave = (size_t(blockIdx.x) * kThreads + threadIdx.x) >> 6;
    const size_t nwaves = (size_t(gridDim.x) * kThreads) >> 6;
    for (size_t b = wave; b < kFloats / 64; b += nwaves) {
        __builtin_amdgcn_global_load_lds(s + b * 64 + lane, (lds_ptr_t)(buf + w * 64), 4, 0, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        acc += buf[w * 64 + lane];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    if (acc == 12345.f) out[threadIdx.x] = acc;
}

__global__ __launch_bounds__(kThreads) void wr_dword(float* __restrict__ d) {
    const size_t stride = size_t(gridDim.x) * kThreads;
    for (size_t i = size_t(blockIdx.x) * kThreads + threadIdx.x; i < kFloats; i += stride) d[i] = 1.f;
}

__global__ __launch_bounds__(kThreads) void wr_dwordx4(float4* __restrict__ d) {
    const size_t stride = size_t(gridDim.x) * kThreads;
    for (size_t i = size_t(blockIdx.x) * kThreads + threadIdx.x; i < kFloats / 4; i += stride)
        d[i] = float4{1.f, 1.f, 1.f, 1.f};
}

__global__ __launch_bounds__(kThreads) void wr_frag(float* __restrict__ d) {
    const int lane = threadIdx.x & 63, krow = lane >> 4, kcol = lane & 15;
    const size_t wave = (size_t(blockIdx.x) * kThreads + threadIdx.x) >> 6;
    const size_t nwaves = (size_t(gridDim.x) * kThreads) >> 6;
    for (size_t b = wave; b < kFloats / 256; b += nwaves) {
        float* p = d + b * 256 + krow * 64 + kcol;
#pragma unroll
        for (int j = 0; j < 4; ++j) p[j * 16] = 1.f;
    }
}

#define CHECK(x)                                                                       \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

}  // namespace

int main() {
    float *src = nullptr, *dst = nullptr, *out = nullptr;
    CHECK(hipMalloc(&src, kFloats * sizeof(float)));
    CHECK(hipMalloc(&dst, kFloats * sizeof(float)));
    CHECK(hipMalloc(&out, kThreads * sizeof(float)));
    CHECK(hipMemset(src, 0, kFloats * sizeof(float)));
    CHECK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    auto run = [&](const char* name, auto&& launch) -> int {
        CHECK(hipEventRecord(e0));
        launch();
        CHECK(hipGetLastError());
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms = 0.f;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-11s 1 GiB in %.3f ms = %.0f GB/s\n", name, ms, kFloats * 4.0 / (ms * 1e6));
        return 0;
    };
    const dim3 g(kBlocks), b(kThreads);
    int rc = 0;
    rc |= run("rd_dword", [&] { hipLaunchKernelGGL(rd_dword, g, b, 0, 0, src, out); });
    rc |= run("rd_dwordx2", [&] { hipLaunchKernelGGL(rd_dwordx2, g, b, 0, 0, (const double*)src, out); });
    rc |= run("rd_dwordx4", [&] { hipLaunchKernelGGL(rd_dwordx4, g, b, 0, 0, (const float4*)src, out); });
    rc |= run("rd_frag", [&] { hipLaunchKernelGGL(rd_frag, g, b, 0, 0, src, out); });
    rc |= run("rd_ldsdma", [&] { hipLaunchKernelGGL(rd_ldsdma, g, b, 0, 0, src, out); });
    rc |= run("wr_dword", [&] { hipLaunchKernelGGL(wr_dword, g, b, 0, 0, dst); });
    rc |= run("wr_dwordx4", [&] { hipLaunchKernelGGL(wr_dwordx4, g, b, 0, 0, (float4*)dst); });
    rc |= run("wr_frag", [&] { hipLaunchKernelGGL(wr_frag, g, b, 0, 0, dst); });
    CHECK(hipFree(src));
    CHECK(hipFree(dst));
    CHECK(hipFree(out));
    return rc;
}
