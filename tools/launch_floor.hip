// launch_floor.hip -- microbenchmark: per-kernel cost of back-to-back
// dependent launches (eager and hipGraph) on one stream, by grid size.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
__global__ void k_empty(int *p) { if (threadIdx.x == 0 && blockIdx.x == 0 && p[0] == 12345) p[1] = 1; }
int main() {
    int *d; (void)hipMalloc(&d, 64); (void)hipMemset(d, 0, 64);
    hipStream_t s; (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    for (int grid : {1, 256, 1024, 4096}) {
        const int N = 200;
        // eager
        for (int i = 0; i < 50; i++) hipLaunchKernelGGL(k_empty, dim3(grid), dim3(256), 0, s, d);
        (void)hipStreamSynchronize(s);
        (void)hipEventRecord(a, s);
        for (int i = 0; i < N; i++) hipLaunchKernelGGL(k_empty, dim3(grid), dim3(256), 0, s, d);
        (void)hipEventRecord(b, s); (void)hipEventSynchronize(b);
        float ms; (void)hipEventElapsedTime(&ms, a, b);
        // graph
        hipGraph_t g; hipGraphExec_t ge;
        (void)hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
        for (int i = 0; i < N; i++) hipLaunchKernelGGL(k_empty, dim3(grid), dim3(256), 0, s, d);
        (void)hipStreamEndCapture(s, &g);
        (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
        (void)hipGraphLaunch(ge, s); (void)hipStreamSynchronize(s);
        (void)hipEventRecord(a, s);
        for (int r = 0; r < 5; r++) (void)hipGraphLaunch(ge, s);
        (void)hipEventRecord(b, s); (void)hipEventSynchronize(b);
        float ms2; (void)hipEventElapsedTime(&ms2, a, b);
        printf("grid %5d: eager %.2f us/kernel, graph %.2f us/kernel\n", grid, ms * 1e3 / N, ms2 * 1e3 / (5 * N));
        (void)hipGraphExecDestroy(ge); (void)hipGraphDestroy(g);
    }
    return 0;
}
