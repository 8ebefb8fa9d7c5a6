// FETCH_SIZE calibration for the perturber kernels' load patterns (MI355X_MICROARCH.md: "other access widths are
// uncalibrated: calibrate on a known byte count in your own access pattern"). A [R][S] fp32 table of 768 MB (past
// the 256 MiB Infinity Cache, so every line is a compulsory HBM read) is read once by
//   P0: wide coalesced streaming, 16 B per lane, 1 KB contiguous per wave instruction (the guide's reference case)
//   P1: the split-bf16 weight gradient's (pert::k_wgrad_bx3) operand loads: lane (a, g) reads row 16i + a at
//       points n0 + 8g and n0 + 8g + 4 (two 16-B loads; 4 lanes x 2 loads = one 128-B line per row and step)
//   P2: the hidden-layer kernels' (pert::k_*_mid_mf) activation loads: lane (a, g) reads row 4s + g at points
//       n0 + 4a .. n0 + 4a + 3 (16 lanes x 16 B = 256 contiguous bytes per row per instruction)
// Each thread adds what it loaded and writes one float. Run under rocprofv3 --pmc FETCH_SIZE and compare
// FETCH_SIZE (KB per launch) with the table's 768 MB.
//   hipcc -O3 --offload-arch=gfx950 -o fetch_calib fetch_calib.hip && rocprofv3 --pmc FETCH_SIZE -- ./fetch_calib
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int R = 192;                  // rows (channels)
constexpr long long S = 1LL << 20;      // points per row: 192 x 1M x 4 B = 768 MB

__global__ __launch_bounds__(256) void k_p0(const float* __restrict__ t, float* __restrict__ out) {
  const long long n = (long long)R * S / 4;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
    acc += ((const f32x4*)t)[i];
  out[blockIdx.x * 256 + threadIdx.x] = acc[0] + acc[1] + acc[2] + acc[3];
}

// P1: a wave owns row tile i (16 rows) and walks the points in 32-point steps; waves over (row tile, point chunk)
__global__ __launch_bounds__(256) void k_p1(const float* __restrict__ t, float* __restrict__ out) {
  const int lane = threadIdx.x & 63, a = lane & 15, g = lane >> 4;
  const int wave = blockIdx.x * 4 + (threadIdx.x >> 6), nw = gridDim.x * 4;
  const int tiles = R / 16;
  const long long chunk = S / (nw / tiles);
  const int tile = wave % tiles;
  const long long c0 = (long long)(wave / tiles) * chunk;
  const float* row = t + (long long)(16 * tile + a) * S;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (long long n0 = c0; n0 < c0 + chunk; n0 += 32) {
    acc += *(const f32x4*)(row + n0 + 8 * g);
    acc += *(const f32x4*)(row + n0 + 8 * g + 4);
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc[0] + acc[1] + acc[2] + acc[3];
}

// P2: a wave owns 4 rows x 64 points per instruction (rows 4s + g), walks its point chunk in 64-point steps
__global__ __launch_bounds__(256) void k_p2(const float* __restrict__ t, float* __restrict__ out) {
  const int lane = threadIdx.x & 63, a = lane & 15, g = lane >> 4;
  const int wave = blockIdx.x * 4 + (threadIdx.x >> 6), nw = gridDim.x * 4;
  const int quads = R / 4;
  const long long chunk = S / (nw / quads);
  const int quad = wave % quads;
  const long long c0 = (long long)(wave / quads) * chunk;
  const float* row = t + (long long)(4 * quad + g) * S;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (long long n0 = c0; n0 < c0 + chunk; n0 += 64) acc += *(const f32x4*)(row + n0 + 4 * a);
  out[blockIdx.x * 256 + threadIdx.x] = acc[0] + acc[1] + acc[2] + acc[3];
}

int main() {
  float *t, *out;
  const size_t bytes = sizeof(float) * R * S;
  if (hipMalloc(&t, bytes) != hipSuccess || hipMalloc(&out, 4096 * 256 * sizeof(float)) != hipSuccess) return 1;
  hipMemset(t, 0, bytes);
  const int grid = 3072;   // 12288 waves: divisible by 12 row tiles (P1) and 48 row quads (P2)
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(k_p0, dim3(grid), dim3(256), 0, 0, t, out);
    hipLaunchKernelGGL(k_p1, dim3(grid), dim3(256), 0, 0, t, out);
    hipLaunchKernelGGL(k_p2, dim3(grid), dim3(256), 0, 0, t, out);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("table %.1f MB; compare FETCH_SIZE (KB) per launch of k_p0 / k_p1 / k_p2\n", bytes / 1e6);
  hipFree(t);
  hipFree(out);
  return 0;
}
