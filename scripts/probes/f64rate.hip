// Micro-probe: issue throughput of fp64 VALU instructions on gfx950 (cycles per
// wave instruction), 8 independent chains per lane, 8 waves per CU.
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHAINS 8
template <int OP>
__global__ __launch_bounds__(256) void probe(double* out, int iters) {
    double v[CHAINS];
#pragma unroll
    for (int j = 0; j < CHAINS; ++j) v[j] = 1.0 + threadIdx.x * 1e-6 + j * 1e-3;
    const double b = 1.0000001, cst = 1e-9;
    int iv[CHAINS];
#pragma unroll
    for (int j = 0; j < CHAINS; ++j) iv[j] = j;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < CHAINS; ++j) {
            if (OP == 0) v[j] = fma(v[j], b, cst);
            if (OP == 1) v[j] = v[j] * b;
            if (OP == 2) v[j] = fmin(v[j], b + j);
            if (OP == 3) v[j] = rint(v[j]) + 0.25;          // rndne + add
            if (OP == 4) v[j] = ldexp(v[j], iv[j] & 1);
            if (OP == 5) { iv[j] += (int)v[j]; }            // cvt_i32_f64
            if (OP == 6) v[j] = __builtin_amdgcn_rsq(v[j]);
            if (OP == 7) v[j] = (double)__builtin_amdgcn_rsqf((float)v[j]);   // cvt f32 + rsq f32 + cvt f64
            if (OP == 8) v[j] = v[j] + b;
        }
    }
    double s = 0;
#pragma unroll
    for (int j = 0; j < CHAINS; ++j) s += v[j] + iv[j];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int OP>
float run(double* out, int iters) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    hipLaunchKernelGGL(probe<OP>, dim3(512), dim3(256), 0, 0, out, iters);
    hipEventRecord(a);
    hipLaunchKernelGGL(probe<OP>, dim3(512), dim3(256), 0, 0, out, iters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    return ms;
}

int main() {
    double* out; hipMalloc(&out, 512 * 256 * 8);
    int dev; hipGetDevice(&dev); int cus; hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    int clk; hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev);   // kHz
    const int iters = 4096;
    const char* names[] = {"fma_f64", "mul_f64", "min_f64", "rndne+add_f64", "ldexp_f64", "cvt_i32_f64+add_u32",
                           "rsq_f64", "cvt_f32+rsq_f32+cvt_f64", "add_f64"};
    float ms[9] = {run<0>(out, iters), run<1>(out, iters), run<2>(out, iters), run<3>(out, iters), run<4>(out, iters),
                   run<5>(out, iters), run<6>(out, iters), run<7>(out, iters), run<8>(out, iters)};
    // wave-instructions per SIMD: 512 blocks x 4 waves / (cus x 4 SIMDs) x iters x CHAINS
    const double winst = 512.0 * 4 / (cus * 4.0) * iters * CHAINS;
    for (int i = 0; i < 9; ++i)
        printf("%-26s %.3f ms  %.2f cycles per wave instruction (clock %d MHz)\n", names[i], ms[i],
               ms[i] * 1e-3 * clk * 1e3 / winst, clk / 1000);
    return 0;
}
