// FETCH_SIZE calibration on gfx950 (MI355X_MICROARCH.md HBM section: "calibrate on a known byte
// count in your own access pattern").  Each kernel reads a 768 MiB buffer (past the 256 MiB
// Infinity Cache) exactly once with one of the access patterns of this repository's kernels and
// writes one float per block, so the algorithmic read bytes are known exactly:
//   k16  : 16 B per lane, fully coalesced (f32x4 streaming; bn / reduce / adam kernels)
//   k8   : 8 B per lane, fully coalesced (bf16x4 operand loads of the weight-GEMMs, opload.h ld4_raw)
//   k4   : 4 B per lane, fully coalesced
//   seg64: 16 B per lane, but a wave reads 64-B halves of 128-B lines (4 lanes per pixel row, as the
//          halo gathers' window loads of a 32-channel bf16 chunk from a 64-channel tensor); the other
//          halves are read by a second pass over the buffer's odd halves, so every byte is read once
// Run:  rocprofv3 --pmc FETCH_SIZE --output-format csv -d <dir> -o run -- ./fetch_calib
// and compare FETCH_SIZE (KiB) per dispatch with the printed byte counts (tools/calib/fetch_calib.py).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

__global__ void k16(const f32x4* __restrict__ p, long long n, float* out) {
  float s = 0.f;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const f32x4 v = p[i];
    s += v[0] + v[1] + v[2] + v[3];
  }
  if (s == 12345.f) out[blockIdx.x] = s;  // data-dependent store keeps the loads
}
__global__ void k8(const f32x2* __restrict__ p, long long n, float* out) {
  float s = 0.f;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const f32x2 v = p[i];
    s += v[0] + v[1];
  }
  if (s == 12345.f) out[blockIdx.x] = s;
}
__global__ void k4(const float* __restrict__ p, long long n, float* out) {
  float s = 0.f;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    s += p[i];
  if (s == 12345.f) out[blockIdx.x] = s;
}
// half: 0 = the first 64 B of every 128-B line, 1 = the second
__global__ void seg64(const f32x4* __restrict__ p, long long nlines, int half, float* out) {
  float s = 0.f;
  const long long nq = nlines * 4;  // 16-B quads per half-line set
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < nq; i += (long long)gridDim.x * blockDim.x) {
    const long long line = i >> 2, q = i & 3;
    const f32x4 v = p[line * 8 + half * 4 + q];
    s += v[0] + v[1] + v[2] + v[3];
  }
  if (s == 12345.f) out[blockIdx.x] = s;
}

int main() {
  const size_t bytes = 768ull << 20;
  void* buf;
  float* out;
  if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 1 << 20) != hipSuccess) return 1;
  hipMemset(buf, 0, bytes);
  hipDeviceSynchronize();
  const dim3 grid(4096), blk(256);
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(k16, grid, blk, 0, 0, (const f32x4*)buf, (long long)(bytes / 16), out);
    hipLaunchKernelGGL(k8, grid, blk, 0, 0, (const f32x2*)buf, (long long)(bytes / 8), out);
    hipLaunchKernelGGL(k4, grid, blk, 0, 0, (const float*)buf, (long long)(bytes / 4), out);
    hipLaunchKernelGGL(seg64, grid, blk, 0, 0, (const f32x4*)buf, (long long)(bytes / 128), 0, out);
    hipLaunchKernelGGL(seg64, grid, blk, 0, 0, (const f32x4*)buf, (long long)(bytes / 128), 1, out);
  }
  hipDeviceSynchronize();
  printf("bytes_read k16 %zu k8 %zu k4 %zu seg64 %zu (each half pass)\n", bytes, bytes, bytes, bytes / 2);
  hipFree(buf);
  hipFree(out);
  return 0;
}
