// v_permlane32_swap semantics probe: out[l] = the value other_half() returns in lane l
// for v = lane id (expected: l ^ 32), with the call under a divergent branch too.
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ double other_half(double v) {
    const unsigned long long u = __double_as_longlong(v);
    const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)u, (unsigned)u, true, false);
    const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(u >> 32), (unsigned)(u >> 32), true, false);
    const bool low = (threadIdx.x & 32) == 0;
    const unsigned plo = low ? lo[1] : lo[0], phi = low ? hi[1] : hi[0];
    return __longlong_as_double(((unsigned long long)phi << 32) | plo);
}

__global__ void k(double* out, double* out2) {
    const int l = threadIdx.x;
    out[l] = other_half((double)l + 0.25);
    const double o = other_half((double)l + 0.5);
    out2[l] = (l % 3 == 0) ? (double)l : o;
}

int main() {
    double *d, *d2, h[64], h2[64];
    hipMalloc(&d, 64 * sizeof(double));
    hipMalloc(&d2, 64 * sizeof(double));
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, d2);
    hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    hipMemcpy(h2, d2, sizeof h2, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; ++l) {
        if (h[l] != (double)(l ^ 32) + 0.25) ++bad;
        if (h2[l] != ((l % 3 == 0) ? (double)l : (double)(l ^ 32) + 0.5)) ++bad;
    }
    printf("permlane32_swap other_half: %s (lane 0 -> %g, lane 40 -> %g)\n", bad ? "WRONG" : "ok", h[0], h[40]);
    return bad ? 1 : 0;
}
