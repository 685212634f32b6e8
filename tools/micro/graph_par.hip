// Do independent branches of a captured hipGraph run concurrently on gfx950 /
// ROCm 7?  Two kernels of 64 workgroups that each spin ~T us, (a) back to back
// on one stream, (b) forked onto a second stream under capture (event fork /
// join), (c) the same graph replayed; prints wall times by HIP events.
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void spin(unsigned long long cycles, unsigned int *out) {
    const unsigned long long t0 = wall_clock64();
    while (wall_clock64() - t0 < cycles) __builtin_amdgcn_s_sleep(2);
    if (threadIdx.x == 0) atomicAdd(out, 1u);
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main() {
    int rate = 0;
    CK(hipDeviceGetAttribute(&rate, hipDeviceAttributeWallClockRate, 0));   // kHz
    const unsigned long long cyc = (unsigned long long)rate * 50 / 1000;     // 50 us
    unsigned int *d;
    CK(hipMalloc(&d, 4));
    hipStream_t s, s2;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    hipEvent_t a, b, f, j;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventCreateWithFlags(&f, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&j, hipEventDisableTiming));
    float ms;
    for (int rep = 0; rep < 3; rep++) {
        // (a) serial, one stream
        CK(hipEventRecord(a, s));
        hipLaunchKernelGGL(spin, dim3(64), dim3(64), 0, s, cyc, d);
        hipLaunchKernelGGL(spin, dim3(64), dim3(64), 0, s, cyc, d);
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        CK(hipEventElapsedTime(&ms, a, b));
        printf("eager one stream: %.1f us\n", ms * 1e3);
        // (b) eager fork / join on two streams
        CK(hipEventRecord(a, s));
        CK(hipEventRecord(f, s));
        CK(hipStreamWaitEvent(s2, f, 0));
        hipLaunchKernelGGL(spin, dim3(64), dim3(64), 0, s, cyc, d);
        hipLaunchKernelGGL(spin, dim3(64), dim3(64), 0, s2, cyc, d);
        CK(hipEventRecord(j, s2));
        CK(hipStreamWaitEvent(s, j, 0));
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        CK(hipEventElapsedTime(&ms, a, b));
        printf("eager two streams: %.1f us\n", ms * 1e3);
        // (c) the fork / join captured into a graph, replayed
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        CK(hipEventRecord(f, s));
        CK(hipStreamWaitEvent(s2, f, 0));
        for (int k = 0; k < 4; k++) {   // two chains of 4 kernels each
            hipLaunchKernelGGL(spin, dim3(64), dim3(64), 0, s, cyc, d);
            hipLaunchKernelGGL(spin, dim3(64), dim3(64), 0, s2, cyc, d);
        }
        CK(hipEventRecord(j, s2));
        CK(hipStreamWaitEvent(s, j, 0));
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        for (int r = 0; r < 2; r++) {
            CK(hipEventRecord(a, s));
            CK(hipGraphLaunch(ge, s));
            CK(hipEventRecord(b, s));
            CK(hipEventSynchronize(b));
            CK(hipEventElapsedTime(&ms, a, b));
            printf("graph, two chains of 4 x 50 us: %.1f us (serial would be 400)\n", ms * 1e3);
        }
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
        // (d) per-edge cost: graphs of short kernels (5 us), one chain of 16 on one stream vs
        // two chains of 8 (fork / join)
        const unsigned long long c5 = (unsigned long long)rate * 5 / 1000;
        for (int two = 0; two < 2; two++) {
            CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
            if (two) {
                CK(hipEventRecord(f, s));
                CK(hipStreamWaitEvent(s2, f, 0));
            }
            for (int k = 0; k < (two ? 8 : 16); k++) {
                hipLaunchKernelGGL(spin, dim3(64), dim3(64), 0, s, c5, d);
                if (two) hipLaunchKernelGGL(spin, dim3(64), dim3(64), 0, s2, c5, d);
            }
            if (two) {
                CK(hipEventRecord(j, s2));
                CK(hipStreamWaitEvent(s, j, 0));
            }
            CK(hipStreamEndCapture(s, &g));
            CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
            for (int r = 0; r < 3; r++) {
                CK(hipEventRecord(a, s));
                CK(hipGraphLaunch(ge, s));
                CK(hipEventRecord(b, s));
                CK(hipEventSynchronize(b));
                CK(hipEventElapsedTime(&ms, a, b));
                if (r) printf("graph of 16 x 5 us kernels, %s: %.1f us\n", two ? "two chains of 8 (ideal 40 + edges)" : "one chain (80 + edges)", ms * 1e3);
            }
            CK(hipGraphExecDestroy(ge));
            CK(hipGraphDestroy(g));
        }
    }
    return 0;
}
