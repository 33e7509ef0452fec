// Probe: can a captured hipGraph carry event-record nodes usable with hipEventElapsedTime?
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void spin(int n, int* x) { int s = 0; for (int i = 0; i < n; i++) s += i ^ threadIdx.x; if (s == 42) *x = s; }
#define CK(c) do { hipError_t e = (c); printf("%-60s -> %s\n", #c, hipGetErrorString(e)); } while (0)
int main() {
  hipStream_t st; CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  int* x; CK(hipMalloc(&x, 4));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  // 1. event record inside capture
  hipGraph_t g; hipGraphExec_t ge;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
  CK(hipEventRecord(a, st));
  hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, st, 1 << 20, x);
  CK(hipEventRecord(b, st));
  CK(hipStreamEndCapture(st, &g));
  CK(hipGetLastError());
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(ge, st));
  CK(hipStreamSynchronize(st));
  float ms = -1; CK(hipEventElapsedTime(&ms, a, b)); printf("captured-record elapsed %f ms\n", ms);
  // 2. explicit event-record nodes
  hipGraph_t g2; CK(hipGraphCreate(&g2, 0));
  hipGraphNode_t n0, n1, n2;
  CK(hipGraphAddEventRecordNode(&n0, g2, nullptr, 0, a));
  hipKernelNodeParams kp = {}; int n = 1 << 20; void* args[] = {&n, &x};
  kp.func = (void*)spin; kp.gridDim = dim3(1); kp.blockDim = dim3(64); kp.kernelParams = args;
  CK(hipGraphAddKernelNode(&n1, g2, &n0, 1, &kp));
  CK(hipGraphAddEventRecordNode(&n2, g2, &n1, 1, b));
  hipGraphExec_t ge2; CK(hipGraphInstantiate(&ge2, g2, nullptr, nullptr, 0));
  CK(hipGraphLaunch(ge2, st)); CK(hipStreamSynchronize(st));
  ms = -1; CK(hipEventElapsedTime(&ms, a, b)); printf("explicit-node elapsed %f ms\n", ms);
  // 3. eager reference
  CK(hipEventRecord(a, st)); hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, st, 1 << 20, x); CK(hipEventRecord(b, st));
  CK(hipStreamSynchronize(st)); ms = -1; CK(hipEventElapsedTime(&ms, a, b)); printf("eager elapsed %f ms\n", ms);
  return 0;
}
