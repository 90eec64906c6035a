// Microbenchmark (diagnostic, not part of the product): issue cost per wave
// instruction of v_add_f32 / v_mul_f32 vs v_pk_add_f32 / v_pk_mul_f32 with
// independent accumulators, at 1..4 waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float v2f __attribute__((ext_vector_type(2)));

template <int MODE>
__global__ void k(float *out, int iters, long long *cyc) {
  float a[16];
  v2f p[8];
  for (int i = 0; i < 16; i++) a[i] = threadIdx.x * 0.001f + i;
  for (int i = 0; i < 8; i++) p[i] = (v2f){a[2 * i], a[2 * i + 1]};
  const float m = out[0] * 1e-30f + 1.0f;
  const v2f mm = (v2f){m, m};
  long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; it++) {
    if (MODE == 0) {
#pragma unroll
      for (int i = 0; i < 16; i++) asm volatile("v_add_f32 %0, %0, %1" : "+v"(a[i]) : "v"(m));
    } else if (MODE == 1) {
#pragma unroll
      for (int i = 0; i < 8; i++) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(p[i]) : "v"(mm));
    } else if (MODE == 2) {
#pragma unroll
      for (int i = 0; i < 8; i++) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(p[i]) : "v"(mm));
    } else {
#pragma unroll
      for (int i = 0; i < 16; i++) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a[i]) : "v"(m));
    }
  }
  long long t1 = __builtin_readcyclecounter();
  float s = 0;
  for (int i = 0; i < 16; i++) s += a[i];
  for (int i = 0; i < 8; i++) s += p[i].x + p[i].y;
  out[blockIdx.x * blockDim.x + threadIdx.x + 1] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

int main() {
  float *out;
  long long *cyc;
  hipMalloc(&out, 1 << 24);
  hipMalloc(&cyc, 8);
  hipMemset(out, 0, 1 << 24);
  const int iters = 4096;
  for (int waves = 1; waves <= 8; waves *= 2) {
    for (int mode = 0; mode < 4; mode++) {
      // one workgroup per CU, `waves` waves per SIMD
      auto kern = mode == 0 ? k<0> : mode == 1 ? k<1> : mode == 2 ? k<2> : k<3>;
      hipLaunchKernelGGL(kern, dim3(256), dim3(64 * 4 * waves), 0, 0, out, iters, cyc);
      hipDeviceSynchronize();
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      hipEventRecord(e0);
      hipLaunchKernelGGL(kern, dim3(256), dim3(64 * 4 * waves), 0, 0, out, iters, cyc);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      long long c;
      hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
      const int ninst = mode == 1 || mode == 2 ? 8 : 16;
      const char *nm[4] = {"v_add_f32", "v_pk_add_f32", "v_pk_mul_f32", "v_mul_f32"};
      // lane-flops per SIMD per cycle implied by the wall time (2.4 GHz nominal)
      const double ops = 256.0 * 4 * waves * 64 * (double)iters * ninst * (mode == 1 || mode == 2 ? 2 : 1);
      printf("waves/SIMD %d %-13s cyc/instr(wave0 counter) %.2f  chip %.1f Tlane-op/s\n", waves, nm[mode],
             (double)c / ((double)iters * ninst), ops / (ms * 1e-3) / 1e12);
    }
  }
  return 0;
}
