// Probes: (1) ds_read_b64_tr_b16 lane mapping, (2) mfma_f32_32x32x16_bf16 C/D layout.
#include <hip/hip_runtime.h>
#include <stdint.h>
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;
extern "C" __global__ void probe_tr(int* out) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[16 * 64];   // [16 rows][64 cols]
  for (int i = threadIdx.x; i < 16 * 64; i += 64) lds[i] = (uint16_t)i;  // value = row*64 + col
  __syncthreads();
  const int l = threadIdx.x, g = l >> 4, i = l & 15, q = i >> 2, p = i & 3;
  // lane 4q+p supplies row (4g + q), cols 4p..4p+3
  const uint16_t* a = lds + (4 * g + q) * 64 + 4 * p;
  s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)a);
  for (int e = 0; e < 4; ++e) out[l * 4 + e] = (uint16_t)v[e];
}
extern "C" __global__ void probe_mfma(float* out) {
  const int l = threadIdx.x, r = l & 31, h = l >> 5;
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    const int k = 8 * h + j;   // assumed k index of element j
    a[j] = (__bf16)(r == k ? 1.0f : 0.0f);              // A[r][k] = delta
    b[j] = (__bf16)(float)(k * 32 + r);                 // B[k][c=r] = k*32 + c
  }
  f32x16 d = {};
  d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, d, 0, 0, 0);
  for (int e = 0; e < 16; ++e) out[l * 16 + e] = d[e];
}
extern "C" int run_probes(int* tr_out, float* mf_out) {
  int *dt; float *dm;
  hipMalloc(&dt, 64 * 4 * 4); hipMalloc(&dm, 64 * 16 * 4);
  probe_tr<<<1, 64>>>(dt); probe_mfma<<<1, 64>>>(dm);
  hipMemcpy(tr_out, dt, 64 * 4 * 4, hipMemcpyDeviceToHost);
  hipMemcpy(mf_out, dm, 64 * 16 * 4, hipMemcpyDeviceToHost);
  hipFree(dt); hipFree(dm);
  return (int)hipGetLastError();
}
