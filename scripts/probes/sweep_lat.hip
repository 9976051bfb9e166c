// Micro-probe: latency of one 32x32 pivot-block sweep (gp_fit.hip's
// pivot_block_sweep_nw) in a single workgroup of 2 / 4 / 8 waves, the form the
// sw_step_kernel workgroups run; plus lower bounds:
// the pivot chain alone (reciprocal + the next pivot's update, 32 times) and a
// barrier + LDS round trip alone.  Shader cycles per sweep (clock64), one
// workgroup per CU on 8 CUs.  Build (scripts/probes/build_sweep_lat.sh):
//   hipcc --offload-arch=gfx950 -O3 -I mpi_opt_amd/csrc sweep_lat.hip -L mpi_opt_amd -lmpo
#include "../../mpi_opt_amd/csrc/gp_fit.hip"
#include <cstdio>

namespace {
template <int MODE, int NW>
__global__ __launch_bounds__(64 * NW) void sweep_lat_kernel(const double* C, double* out, long long* cyc, int reps) {
    __shared__ double rowb[2 * 2 * kSwNb];
    __shared__ double colb[2 * 2 * kSwNb];
    const int wv = threadIdx.x >> 6;
    double acc = 0.0;
    __syncthreads();
    const long long t0 = clock64();
    for (int it = 0; it < reps; ++it) {
        constexpr int CW = 16 / NW;
        double r[CW], prod = 1.0;
        int bad = 0;
        if (MODE == 0) pivot_block_sweep_nw<NW>(C, 0, rowb, colb, wv, r, prod, bad);
        if (MODE == 2) {   // the serial pivot chain alone: 32 x (rcp chain, one fma)
            double pv = C[threadIdx.x & 31] + 2.0;
#pragma unroll
            for (int c = 0; c < kSwNb; ++c) {
                const double ip = pivot_rcp(pv);
                pv = fma(-ip, 0.25, pv + 1.0);
                prod *= pv;
            }
#pragma unroll
            for (int jj = 0; jj < CW; ++jj) r[jj] = pv;
        }
        if (MODE == 3) {   // 16 barrier + LDS round trips alone
            double v = C[threadIdx.x & 31];
#pragma unroll
            for (int c = 0; c < kSwNb; c += 2) {
                double* rb = rowb + ((c >> 1) & 1) * 64;
                if ((threadIdx.x & 63) == c) rb[0] = v;
                __syncthreads();
                v += rb[0];
            }
#pragma unroll
            for (int jj = 0; jj < CW; ++jj) r[jj] = v;
        }
#pragma unroll
        for (int jj = 0; jj < CW; ++jj) acc += r[jj];
        acc += prod + bad;
        __syncthreads();
    }
    const long long t1 = clock64();
    out[blockIdx.x * 512 + threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
}  // namespace

int main() {
    // an SPD 32x32 block: K = I*4 + small symmetric coupling, row-major [32][32]
    double h[32 * 32];
    for (int i = 0; i < 32; ++i)
        for (int j = 0; j < 32; ++j) h[i * 32 + j] = i == j ? 4.0 : 0.5 / (1 + (i > j ? i - j : j - i));
    double *C, *out;
    long long* cyc;
    hipMalloc(&C, sizeof(h));
    hipMalloc(&out, 8 * 512 * sizeof(double));
    hipMalloc(&cyc, 8 * sizeof(long long));
    hipMemcpy(C, h, sizeof(h), hipMemcpyHostToDevice);
    const char* names[6] = {"sweep, 2 waves", "sweep, 4 waves", "sweep, 8 waves", "",
                            "pivot chain alone (32 x rcp + fma)", "16 barrier + LDS round trips"};
    const int reps = 2000;
    for (int pass = 0; pass < 2; ++pass)
        for (int mode = 0; mode < 6; ++mode) {
            if (mode == 0) hipLaunchKernelGGL((sweep_lat_kernel<0, 2>), dim3(8), dim3(128), 0, 0, C, out, cyc, reps);
            if (mode == 1) hipLaunchKernelGGL((sweep_lat_kernel<0, 4>), dim3(8), dim3(256), 0, 0, C, out, cyc, reps);
            if (mode == 2) hipLaunchKernelGGL((sweep_lat_kernel<0, 8>), dim3(8), dim3(512), 0, 0, C, out, cyc, reps);
            if (mode == 3) continue;
            if (mode == 4) hipLaunchKernelGGL((sweep_lat_kernel<2, 4>), dim3(8), dim3(256), 0, 0, C, out, cyc, reps);
            if (mode == 5) hipLaunchKernelGGL((sweep_lat_kernel<3, 4>), dim3(8), dim3(256), 0, 0, C, out, cyc, reps);
            long long c[8];
            hipMemcpy(c, cyc, sizeof(c), hipMemcpyDeviceToHost);
            if (pass == 1) printf("%-40s %8.0f shader cycles per sweep\n", names[mode], (double)c[0] / reps);
        }
    return 0;
}
