// Dependent kernel boundary on one stream (MI355X_MICROARCH.md "boundary" row), measured on the box:
//   k launches of a kernel that spins S ns and writes W bytes, vs ONE launch spinning k*S ns and
//   writing k*W bytes: the difference per launch is the boundary (dispatch + completion + release
//   of the W dirty bytes).  Explains the main stream's untraced idle: ~580 dependent launches per
//   training step.   hipcc --offload-arch=gfx950 -O2 boundary.hip -o boundary
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void spin_write(long long ns, float* out, long long nfloat) {
  const long long t0 = wall_clock64();  // 100 MHz constant clock
  const long long ticks = ns / 10;
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(1);
  const long long stride = (long long)gridDim.x * blockDim.x * 4;
  for (long long i = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < nfloat; i += stride)
    *(float4*)(out + i) = make_float4(1.f, 2.f, 3.f, (float)i);
}

static float run(int launches, long long ns, float* buf, long long nfloat, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
  hipEventRecord(e0, s);
  for (int i = 0; i < launches; ++i) hipLaunchKernelGGL(spin_write, dim3(1024), dim3(256), 0, s, ns, buf, nfloat);
  hipEventRecord(e1, s);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  return ms;
}

int main() {
  hipStream_t s;
  hipStreamCreate(&s);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const long long maxb = 256LL << 20;
  float* buf;
  if (hipMalloc(&buf, maxb) != hipSuccess) return 1;
  const int K = 200;
  printf("spin_ns  write_MB  per_launch_us(k=%d)  one_long_launch_us/k  boundary_us\n", K);
  for (long long wmb : {0LL, 4LL, 16LL}) {
    for (long long ns : {0LL, 4000LL, 10000LL}) {
      const long long nf = wmb * (1 << 20) / 4;
      run(20, ns, buf, nf, s, e0, e1);  // warm
      const float many = run(K, ns, buf, nf, s, e0, e1);
      // one launch with K x the spin; its writes: the same W bytes rewritten K times is not K*W of
      // fresh traffic, so the dirty-byte release appears once: boundary includes (K-1) releases
      run(2, ns * K, buf, nf, s, e0, e1);
      const float one = run(1, ns * K, buf, nf, s, e0, e1);
      printf("%7lld  %8lld  %19.3f  %20.3f  %11.3f\n", ns, wmb, many * 1e3 / K, one * 1e3 / K,
             (many - one) * 1e3 / (K - 1));
    }
  }
  hipFree(buf);
  return 0;
}
