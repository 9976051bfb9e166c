// Micro-probe: can fp64 VALU work of one wave execute while another wave's
// fp64 MFMAs run on the same SIMD?  mode 0: MFMA waves only, mode 1: VALU waves
// only, mode 2: both kinds on every SIMD (2 waves per SIMD, one of each).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double f64x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// same experiment in fp32: v_mfma_f32_16x16x4_f32 chains vs fp32 FMA waves
__global__ __launch_bounds__(512) void probe32(float* out, int mode, int iters) {
    const int wave = threadIdx.x >> 6;
    const bool mfma_wave = mode == 0 ? true : (mode == 1 ? false : (wave < 4));
    const bool active = mode == 2 ? true : (wave < 4);
    if (!active) return;
    float a = threadIdx.x * 1e-3f, b = 1.0f + threadIdx.x * 1e-4f;
    if (mfma_wave) {
        f32x4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
        for (int i = 0; i < iters; ++i) {
            c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c3, 0, 0, 0);
        }
        out[blockIdx.x * 512 + threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3];
    } else {
        float v[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = a + j;
        for (int i = 0; i < iters * 4; ++i) {
#pragma unroll
            for (int j = 0; j < 16; ++j) v[j] = fmaf(v[j], b, 1e-9f);
        }
        float s = 0;
#pragma unroll
        for (int j = 0; j < 16; ++j) s += v[j];
        out[blockIdx.x * 512 + threadIdx.x] = s;
    }
}

__global__ __launch_bounds__(512) void probe(double* out, int mode, int iters) {
    const int wave = threadIdx.x >> 6;            // 8 waves: wave w on SIMD w % 4
    const bool mfma_wave = mode == 0 ? true : (mode == 1 ? false : (wave < 4));
    const bool active = mode == 2 ? true : (wave < 4);
    if (!active) return;
    double a = threadIdx.x * 1e-3, b = 1.0 + threadIdx.x * 1e-4;
    if (mfma_wave) {
        f64x4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
        for (int i = 0; i < iters; ++i) {
            c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
        }
        out[blockIdx.x * 512 + threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3];
    } else {
        double v[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = a + j;
        for (int i = 0; i < iters * 4; ++i) {
#pragma unroll
            for (int j = 0; j < 16; ++j) v[j] = fma(v[j], b, 1e-9);
        }
        double s = 0;
#pragma unroll
        for (int j = 0; j < 16; ++j) s += v[j];
        out[blockIdx.x * 512 + threadIdx.x] = s;
    }
}

int main() {
    double* out;
    hipMalloc(&out, 256 * 512 * sizeof(double));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 20000;
    for (int rep = 0; rep < 2; ++rep)
        for (int mode = 0; mode < 3; ++mode) {
            hipLaunchKernelGGL(probe, dim3(256), dim3(512), 0, 0, out, mode, iters);
            hipEventRecord(e0);
            hipLaunchKernelGGL(probe, dim3(256), dim3(512), 0, 0, out, mode, iters);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            const double mfma_cyc = 4.0 * iters;          // MFMAs per MFMA wave
            const double valu_ins = 16.0 * 4 * iters;     // fp64 FMAs per VALU wave
            printf("mode %d (%s): %.3f ms   [%.1f ns per MFMA / %.2f ns per VALU fma, per wave]\n", mode,
                   mode == 0 ? "MFMA only" : mode == 1 ? "VALU only" : "MFMA + VALU waves per SIMD", ms,
                   ms * 1e6 / mfma_cyc, ms * 1e6 / valu_ins);
        }
    for (int rep = 0; rep < 2; ++rep)
        for (int mode = 0; mode < 3; ++mode) {
            hipLaunchKernelGGL(probe32, dim3(256), dim3(512), 0, 0, reinterpret_cast<float*>(out), mode, iters);
            hipEventRecord(e0);
            hipLaunchKernelGGL(probe32, dim3(256), dim3(512), 0, 0, reinterpret_cast<float*>(out), mode, iters);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            printf("fp32 mode %d (%s): %.3f ms\n", mode,
                   mode == 0 ? "MFMA only" : mode == 1 ? "VALU only" : "MFMA + VALU waves per SIMD", ms);
        }
    return 0;
}
