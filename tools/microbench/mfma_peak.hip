// Bare v_mfma_f32_16x16x32_bf16 throughput on this device: every CU runs WAVES waves, each issuing
// ITERS x 32 independent MFMAs from registers (no memory traffic), operands random-ish (lane bits)
// or zero. Calibrates the attainable MFMA rate (clock under load) against the 2.5 PF nominal peak.
//   hipcc -O3 --offload-arch=gfx950 -o mfma_peak mfma_peak.hip && ./mfma_peak
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int ZERO>
__global__ __launch_bounds__(512) void k_mfma(int iters, float* out) {
  const unsigned l = threadIdx.x * 2654435761u + blockIdx.x;
  bf16x8 a[4], b[8];
#pragma unroll
  for (int i = 0; i < 4; ++i) a[i] = ZERO ? (bf16x8){} : __builtin_bit_cast(bf16x8, make_uint4(l * (i + 3), l ^ 0x3c3c3c3c, l + i, l * 7));
#pragma unroll
  for (int j = 0; j < 8; ++j) b[j] = ZERO ? (bf16x8){} : __builtin_bit_cast(bf16x8, make_uint4(l + j, l * 13, l ^ (j * 77), l * 3));
  f32x4 acc[4][8] = {};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) s += acc[i][j][0] + acc[i][j][3];
  if (s == 1.2345f) out[0] = s;
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  float* out;
  hipMalloc(&out, 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 4000;
  for (int zero = 0; zero < 2; ++zero)
    for (int waves : {4, 8}) {
      for (int rep = 0; rep < 3; ++rep) {
        hipEventRecord(e0);
        for (int k = 0; k < 5; ++k) {
          if (zero) hipLaunchKernelGGL(k_mfma<1>, dim3(cus), dim3(64 * waves), 0, 0, iters, out);
          else hipLaunchKernelGGL(k_mfma<0>, dim3(cus), dim3(64 * waves), 0, 0, iters, out);
        }
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        const double flop = 5.0 * cus * waves * (double)iters * 32 * 16384;
        if (rep == 2) printf("zero=%d waves/CU=%d: %.1f TFLOP/s (%.3f of 2.5 PF), %.2f ms\n", zero, waves, flop / (ms * 1e-3) / 1e12,
                             flop / (ms * 1e-3) / 2.5e15, ms);
      }
    }
  return 0;
}
