// Issue rate of the f32-input MFMA forms on gfx950: cycles per instruction per
// wave, back to back on independent accumulators (one wave per SIMD).
//   hipcc --offload-arch=gfx950 -O3 -o mfma_rate mfma_rate.hip && ./mfma_rate
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));

constexpr int kIters = 4096;

__global__ void __launch_bounds__(256) k16x16x4(float* out, long long* cyc, float a, float b) {
    f4 c[4] = {};
    long long t0 = clock64();
    for (int i = 0; i < kIters; ++i) {
#pragma unroll
        for (int j = 0; j < 4; ++j) c[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c[j], 0, 0, 0);
    }
    long long t1 = clock64();
    float s = 0.f;
    for (int j = 0; j < 4; ++j) s += c[j][0] + c[j][1] + c[j][2] + c[j][3];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void __launch_bounds__(256) k4x4x1(float* out, long long* cyc, float a, float b) {
    f4 c[8] = {};
    long long t0 = clock64();
    for (int i = 0; i < kIters; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) c[j] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c[j], 0, 0, 0);
    }
    long long t1 = clock64();
    float s = 0.f;
    for (int j = 0; j < 8; ++j) s += c[j][0] + c[j][1] + c[j][2] + c[j][3];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void __launch_bounds__(256) k16x16x1(float* out, long long* cyc, float a, float b) {
    f16v c[2] = {};
    long long t0 = clock64();
    for (int i = 0; i < kIters; ++i) {
#pragma unroll
        for (int j = 0; j < 2; ++j) c[j] = __builtin_amdgcn_mfma_f32_16x16x1f32(a, b, c[j], 0, 0, 0);
    }
    long long t1 = clock64();
    float s = 0.f;
    for (int j = 0; j < 2; ++j)
        for (int e = 0; e < 16; ++e) s += c[j][e];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <class K>
void run(const char* name, K kern, int per_iter, double flops_per_inst) {
    float* out;
    long long* cyc;
    const int blocks = 256;
    hipMalloc(&out, blocks * 256 * sizeof(float));
    hipMalloc(&cyc, blocks * sizeof(long long));
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, cyc, 1.0f, 0.5f);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, cyc, 1.0f, 0.5f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    long long h[256];
    hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    double mean = 0;
    for (int i = 0; i < blocks; ++i) mean += h[i];
    mean /= blocks;
    const double insts = (double)kIters * per_iter;
    const double tf = flops_per_inst * insts * 4 * blocks / (ms * 1e-3) / 1e12;
    printf("%-22s %6.2f cycles per instruction per wave (clock64), %.1f TF/s chip-wide\n", name, mean / insts, tf);
    hipFree(out);
    hipFree(cyc);
}

// Operand / result layout of v_mfma_f32_4x4x1_16b_f32: lane l supplies a = 1000 + l,
// b = l; each result element should be a(lane of its row) * b(lane of its column).
__global__ void layout4x4(float* out) {
    const int l = threadIdx.x;
    f4 c = {0.f, 0.f, 0.f, 0.f};
    c = __builtin_amdgcn_mfma_f32_4x4x1f32(1000.f + l, (float)l, c, 0, 0, 0);
    for (int i = 0; i < 4; ++i) out[l * 4 + i] = c[i];
}

void layout() {
    float* d;
    hipMalloc(&d, 256 * sizeof(float));
    hipLaunchKernelGGL(layout4x4, dim3(1), dim3(64), 0, 0, d);
    float h[256];
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; ++l)
        for (int i = 0; i < 4; ++i) {
            // hypothesis: block b = l / 4, column j = l % 4, VGPR i = row i; A row i of
            // block b from lane 4b + i, B column j from lane 4b + j
            const int b = l / 4, j = l % 4;
            const float want = (1000.f + 4 * b + i) * (float)(4 * b + j);
            if (h[l * 4 + i] != want) {
                if (bad < 8) printf("lane %d vgpr %d: got %.0f want %.0f\n", l, i, h[l * 4 + i], want);
                ++bad;
            }
        }
    printf("4x4x1_16b layout hypothesis (block = lane/4, col = lane%%4, vgpr = row): %s (%d mismatches)\n",
           bad ? "WRONG" : "confirmed", bad);
    hipFree(d);
}

int main() {
    layout();
    run("v_mfma_f32_16x16x4f32", k16x16x4, 4, 16 * 16 * 4 * 2.0);
    run("v_mfma_f32_4x4x1_16b", k4x4x1, 8, 16 * 4 * 4 * 2.0);
    run("v_mfma_f32_16x16x1_4b", k16x16x1, 2, 4 * 16 * 16 * 2.0);
    return 0;
}
