// BN apply / backward-apply passes at the CelebA step's shapes (the split mode's fp32 tensors), timed alone:
// the engine's grid (2 rows per thread, 32 accumulator shards), more rows per thread, one shard, no shard
// gather at all (statistics already finalised), against a plain 2-read-1-write float4 stream of the same bytes.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I sequential-variational-autoencoder_amd/csrc \
//         tools/calib/bn_micro.hip -o tools/calib/bn_micro
#include "bn.hip"

#include <cstdio>
#include <vector>

__global__ __launch_bounds__(256) void stream3(const float4* a, const float4* b, float4* c, long long n) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const float4 x = a[i], y = b[i];
    c[i] = make_float4(x.x * y.x, x.y + y.y, x.z - y.z, x.w * 0.5f);
  }
}

static ApGrid grid_rpt(long long rows, int C, int groups, int rpt, int capb) {
  const int Q = C / 4, QB = Q < AP_QB ? Q : AP_QB, RL = 256 / QB, gx = (Q + QB - 1) / QB;
  long long want = (rows + (long long)rpt * RL - 1) / ((long long)rpt * RL);
  long long cap = capb / ((long long)gx * groups);
  if (cap < 1) cap = 1;
  long long ry = want < cap ? want : cap;
  if (ry < 1) ry = 1;
  ApGrid g;
  g.rpb = (int)((rows + ry - 1) / ry);
  g.grid = dim3(gx, (unsigned)((rows + g.rpb - 1) / g.rpb), groups);
  return g;
}

int main() {
  struct Shape { long long rows; int C, groups; };
  const Shape shapes[] = {{131072, 32, 1}, {32768, 64, 1}, {8192, 128, 1}, {131072, 32, 8}};
  hipStream_t s;
  hipStreamCreate(&s);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int NIT = 200;
  auto timeit = [&](auto&& fn) {
    for (int i = 0; i < 10; ++i) fn();
    hipEventRecord(e0, s);
    for (int i = 0; i < NIT; ++i) fn();
    hipEventRecord(e1, s);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    return ms * 1e3f / NIT;
  };
  for (const Shape& sh : shapes) {
    const long long n = sh.rows * sh.C * sh.groups;
    float *pre, *dy, *out, *mean, *invstd, *beta, *dbeta, *ab;
    u64* acc;
    const int NSH = 32;
    hipMalloc(&pre, n * 4);
    hipMalloc(&dy, n * 4);
    hipMalloc(&out, n * 4);
    hipMalloc(&mean, sh.C * sh.groups * 4);
    hipMalloc(&invstd, sh.C * sh.groups * 4);
    hipMalloc(&beta, sh.C * sh.groups * 4);
    hipMalloc(&dbeta, sh.C * sh.groups * 4);
    hipMalloc(&ab, 2 * sh.C * sh.groups * 4);
    hipMalloc(&acc, (size_t)NSH * 4 * sh.C * sh.groups * 8);
    std::vector<float> h(n);
    for (long long i = 0; i < n; ++i) h[i] = (float)((i * 2654435761ULL) % 1000) * 1e-3f - 0.5f;
    hipMemcpy(pre, h.data(), n * 4, hipMemcpyHostToDevice);
    hipMemcpy(dy, h.data(), n * 4, hipMemcpyHostToDevice);
    std::vector<float> ones(sh.C * sh.groups, 1.f);
    hipMemcpy(invstd, ones.data(), ones.size() * 4, hipMemcpyHostToDevice);
    hipMemset(mean, 0, sh.C * sh.groups * 4);
    hipMemset(beta, 0, sh.C * sh.groups * 4);
    hipMemset(ab, 0, 2 * sh.C * sh.groups * 4);
    hipMemset(acc, 0, (size_t)NSH * 4 * sh.C * sh.groups * 8);
    const long long acc_gs = (long long)NSH * 4 * sh.C, ssh = 4LL * sh.C;
    const double mb2 = 2.0 * n * 4 / 1e6, mb3 = 3.0 * n * 4 / 1e6;
    printf("rows %lld C %d groups %d (%.1f MB per tensor)\n", sh.rows, sh.C, sh.groups, n * 4 / 1e6);
    const float ts = timeit([&] {
      hipLaunchKernelGGL(stream3, dim3(4096), dim3(256), 0, s, (const float4*)pre, (const float4*)dy, (float4*)out, n / 4);
    });
    printf("  stream 2r1w                       %7.2f us  %6.2f TB/s\n", ts, mb3 / ts);
    const int rpts[] = {2, 4, 8, 16};
    for (int mode = 0; mode < 3; ++mode) {  // 0: 32 shards, 1: one shard, 2: no gather
      for (int rpt : rpts) {
        const ApGrid g = grid_rpt(sh.rows, sh.C, sh.groups, rpt, 4096);
        const int nsh = mode == 1 ? 1 : NSH;
        const u64* a = mode == 2 ? nullptr : acc;
        const float tf = timeit([&] {
          hipLaunchKernelGGL((bn_apply_kernel<4, false>), g.grid, dim3(256), 0, s, pre, sh.C, sh.rows * sh.C, sh.rows, sh.C,
                             a, acc_gs, ssh, nsh, 1e-3f, mean, invstd, (long long)sh.C, beta, (long long)sh.C,
                             (const float*)nullptr, 0, 0LL, 1, out, sh.C, sh.rows * sh.C, g.rpb, 0);
        });
        const float tb = timeit([&] {
          hipLaunchKernelGGL((bn_bwd_apply_kernel<4, false, false>), g.grid, dim3(256), 0, s, dy, sh.C, sh.rows * sh.C,
                             (const float*)nullptr, 0, 0LL, pre, sh.C, sh.rows * sh.C, sh.rows, sh.C, mean, invstd,
                             (long long)sh.C, beta, (long long)sh.C, a, acc_gs, ssh, nsh, dbeta, (long long)sh.C, 1,
                             out, sh.C, sh.rows * sh.C, (float*)nullptr, 0, 0LL, 0, g.rpb, 0,
                             mode == 2 ? (const float*)ab : (const float*)nullptr);
        });
        printf("  %-9s rpt %2d grid (%u,%u,%u): apply %7.2f us %5.2f TB/s | bwd apply %7.2f us %5.2f TB/s\n",
               mode == 0 ? "32 shards" : (mode == 1 ? "1 shard" : "no gather"), rpt, g.grid.x, g.grid.y, g.grid.z, tf,
               mb2 / tf, tb, mb3 / tb);
      }
    }
    hipFree(pre); hipFree(dy); hipFree(out); hipFree(mean); hipFree(invstd); hipFree(beta); hipFree(dbeta);
    hipFree(ab); hipFree(acc);
  }
  const hipError_t e = hipGetLastError();
  printf("%s\n", hipGetErrorString(e));
  return e == hipSuccess ? 0 : 1;
}
