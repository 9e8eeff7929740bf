// Cost of the main stream's side-stream hand-overs: a chain of K dependent 4-us kernels on
// stream A, each handing its output to stream B, where a tiny kernel checks it.  The hand-over is
//   mode 0: none (the chain alone)
//   mode 1: hipEventRecord(ev, A) + hipStreamWaitEvent(B, ev) after each kernel (the engine's on_side / side_flush)
//   mode 2: the kernel launched with hipExtLaunchKernelGGL(..., stopEvent = ev) + hipStreamWaitEvent(B, ev)
//   mode 3: mode 1's records without the B work (the marker alone)
//   mode 4: an empty kernel launched with hipExtLaunchKernelGGL(..., stopEvent = ev) after each kernel (the
//           event rides on a dispatch packet instead of a marker) + hipStreamWaitEvent(B, ev)
//   mode 5: mode 1 without B's kernel (the cross-stream wait alone)
//   mode 6: B's kernel after each A kernel with no dependency (concurrent dispatch alone)
//   mode 7: hipStreamWriteValue32 on A after each kernel, hipStreamWaitValue32 (>=) + the check on B
// Prints the A chain's time per kernel and the number of B checks that saw a stale value (must be 0 for a
// usable hand-over).   hipcc --offload-arch=gfx950 -O2 evmarker.hip -o evmarker
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void spin_put(long long ns, int* flags, int i, float* buf, long long nfloat) {
  const long long t0 = wall_clock64();  // 100 MHz constant clock
  while (wall_clock64() - t0 < ns / 10) __builtin_amdgcn_s_sleep(1);
  const long long stride = (long long)gridDim.x * blockDim.x * 4;
  for (long long k = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4; k < nfloat; k += stride)
    *(float4*)(buf + k) = make_float4(1.f, 2.f, 3.f, (float)i);
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) flags[i] = i + 1;  // (a vector store: one lane, divergent)
}
__global__ void nop() {}
__global__ void check(const int* flags, int i, int* bad) {
  if (threadIdx.x == 0 && __atomic_load_n(&flags[i], __ATOMIC_RELAXED) != i + 1) atomicAdd(bad, 1);
}

int main() {
  hipStream_t A, B;
  hipStreamCreateWithFlags(&A, hipStreamNonBlocking);
  hipStreamCreateWithFlags(&B, hipStreamNonBlocking);
  const int K = 300, R = 16;
  std::vector<hipEvent_t> ev(R);
  for (auto& e : ev) hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventDisableSystemFence);
  hipEvent_t t0, t1;
  hipEventCreate(&t0);
  hipEventCreate(&t1);
  int *flags, *bad;
  void* seq;  // mode 7's sequence word
  if (hipMalloc(&seq, 64) != hipSuccess) return 2;
  float* buf;
  const long long nfloat = 1LL << 20;  // 4 MB written per kernel
  if (hipMalloc(&flags, K * sizeof(int)) != hipSuccess || hipMalloc(&bad, sizeof(int)) != hipSuccess ||
      hipMalloc(&buf, nfloat * 4) != hipSuccess)
    return 1;
  printf("mode  us_per_kernel  stale_checks\n");
  for (int rep = 0; rep < 2; ++rep)
    for (int mode = 0; mode < 8; ++mode) {
      hipMemset(flags, 0, K * sizeof(int));
      hipMemset(bad, 0, sizeof(int));
      hipMemset(seq, 0, 8);
      hipDeviceSynchronize();
      hipEventRecord(t0, A);
      for (int i = 0; i < K; ++i) {
        hipEvent_t e = ev[i % R];
        if (mode == 2)
          hipExtLaunchKernelGGL(spin_put, dim3(1024), dim3(256), 0, A, nullptr, e, 0, 4000LL, flags, i, buf, nfloat);
        else
          hipLaunchKernelGGL(spin_put, dim3(1024), dim3(256), 0, A, 4000LL, flags, i, buf, nfloat);
        if (mode == 1 || mode == 3 || mode == 5) hipEventRecord(e, A);
        if (mode == 4) hipExtLaunchKernelGGL(nop, dim3(1), dim3(64), 0, A, nullptr, e, 0);
        if (mode == 1 || mode == 2 || mode == 4 || mode == 5) hipStreamWaitEvent(B, e, 0);
        if (mode == 7) {
          hipStreamWriteValue32(A, seq, (uint32_t)(i + 1), 0);
          hipStreamWaitValue32(B, seq, (uint32_t)(i + 1), hipStreamWaitValueGte, 0xffffffffu);
        }
        if (mode == 1 || mode == 2 || mode == 4 || mode == 7)
          hipLaunchKernelGGL(check, dim3(1), dim3(64), 0, B, flags, i, bad);
        if (mode == 6) hipLaunchKernelGGL(nop, dim3(1), dim3(64), 0, B);
      }
      hipEventRecord(t1, A);
      hipDeviceSynchronize();
      float ms = 0.f;
      hipEventElapsedTime(&ms, t0, t1);
      int nbad = -1;
      hipMemcpy(&nbad, bad, sizeof(int), hipMemcpyDeviceToHost);
      printf("%4d  %13.3f  %12d\n", mode, ms * 1e3f / K, (mode == 0 || mode == 3 || mode == 5 || mode == 6) ? 0 : nbad);
    }
  return 0;
}
