// Micro-probe: host cost of a kernel launch and launch -> completion latency for a
// 3.3 KB by-value kernel argument (the LML sweep's LmlGroup) against a 64-byte one.
// Empty kernels; hipLaunchKernelGGL call time averaged over back-to-back launches,
// and one launch + hipStreamSynchronize round trip on an idle stream.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

struct Big { int a[16]; double t[40][10]; };
struct Small { int a[16]; };

__global__ void kbig(Big g, int* out) { if (threadIdx.x == 0 && g.a[0] == 12345) out[0] = (int)g.t[3][2]; }
__global__ void ksmall(Small g, int* out) { if (threadIdx.x == 0 && g.a[0] == 12345) out[0] = 1; }

int main() {
    int* out;
    hipMalloc(&out, 64);
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    Big big{};
    Small small{};
    using clk = std::chrono::steady_clock;
    for (int pass = 0; pass < 2; ++pass) {
        for (int which = 0; which < 2; ++which) {
            const int N = 2000;
            hipStreamSynchronize(s);
            auto t0 = clk::now();
            for (int i = 0; i < N; ++i) {
                if (which) hipLaunchKernelGGL(kbig, dim3(64), dim3(256), 0, s, big, out);
                else hipLaunchKernelGGL(ksmall, dim3(64), dim3(256), 0, s, small, out);
            }
            auto t1 = clk::now();
            hipStreamSynchronize(s);
            auto t2 = clk::now();
            // launch + sync round trips on an idle stream
            double rt = 0, call = 0;
            const int R = 500;
            for (int i = 0; i < R; ++i) {
                auto a = clk::now();
                if (which) hipLaunchKernelGGL(kbig, dim3(64), dim3(256), 0, s, big, out);
                else hipLaunchKernelGGL(ksmall, dim3(64), dim3(256), 0, s, small, out);
                auto b = clk::now();
                hipStreamSynchronize(s);
                auto c = clk::now();
                call += std::chrono::duration<double, std::micro>(b - a).count();
                rt += std::chrono::duration<double, std::micro>(c - a).count();
            }
            if (pass == 1)
                printf("%-6s kernarg %5zu B: back-to-back %.2f us per launch call (%.2f us per kernel incl. drain); "
                       "idle-stream launch call %.2f us, launch + sync round trip %.2f us\n",
                       which ? "big" : "small", which ? sizeof(Big) : sizeof(Small),
                       std::chrono::duration<double, std::micro>(t1 - t0).count() / N,
                       std::chrono::duration<double, std::micro>(t2 - t0).count() / N, call / R, rt / R);
        }
    }
    // 100 dependent empty kernels: stream launches vs one hipGraph replay (device-side gap per kernel)
    for (int pass = 0; pass < 2; ++pass) {
        const int K = 100, R = 50;
        hipGraph_t g;
        hipGraphExec_t ge;
        hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
        for (int i = 0; i < K; ++i) hipLaunchKernelGGL(ksmall, dim3(64), dim3(256), 0, s, small, out);
        hipStreamEndCapture(s, &g);
        hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        float ms_stream = 0, ms_graph = 0;
        for (int r = 0; r < R; ++r) {
            hipEventRecord(e0, s);
            for (int i = 0; i < K; ++i) hipLaunchKernelGGL(ksmall, dim3(64), dim3(256), 0, s, small, out);
            hipEventRecord(e1, s);
            hipEventSynchronize(e1);
            float t;
            hipEventElapsedTime(&t, e0, e1);
            ms_stream += t;
            hipEventRecord(e0, s);
            hipGraphLaunch(ge, s);
            hipEventRecord(e1, s);
            hipEventSynchronize(e1);
            hipEventElapsedTime(&t, e0, e1);
            ms_graph += t;
        }
        if (pass == 1)
            printf("100 dependent empty kernels: stream %.2f us per kernel, hipGraph replay %.2f us per kernel\n",
                   ms_stream * 1e3 / (R * K), ms_graph * 1e3 / (R * K));
        hipGraphExecDestroy(ge);
        hipGraphDestroy(g);
    }
    return 0;
}
