// Microbenchmark (diagnostic, not part of the product): the floor of k_prep3's
// serial HP biquad (fvad_staged.hip prep_chain `step`, rnnoise denoise.c
// biquad with f64 intermediates), register-only: a lane walks its own chain
// over samples held in registers, so no memory latency is involved.
//   mode 0  the exact step, 1 chain per lane               (the chain floor)
//   mode 1  + the kernel's side work per sample: the RMS sum (mul + add,
//           unfused) and the y value kept (an add into a checksum)
//   mode 2  2 independent chains per lane, interleaved      (ILP: 2 streams per lane)
//   mode 3  4 independent chains per lane, interleaved
//   mode 4  mode 1's side work with the chain reformulated: b1 * x and the
//           (double)mem1 conversion issued one sample early (off the chain)
// Reported: shader-clock cycles per sample per chain (wave 0's s_memtime),
// at 1 wave per SIMD (one 256-thread workgroup per CU) and 2 waves per SIMD.
// Build: hipcc -O3 -ffp-contract=off --offload-arch=gfx950 biquad.hip -o biquad
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kReg = 32;  // samples held in registers, walked round-robin

template <int MODE>
__global__ void __launch_bounds__(512) kb(const float *in, float *out, int iters, long long *cyc) {
  constexpr int NC = MODE == 2 ? 2 : MODE == 3 ? 4 : 1;
  float x[kReg];
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
#pragma unroll
  for (int i = 0; i < kReg; i++) x[i] = in[(gid * 7 + i) & 4095];
  float mem0[NC], mem1[NC];
#pragma unroll
  for (int c = 0; c < NC; c++) {
    mem0[c] = 0.01f * c;
    mem1[c] = 0.0f;
  }
  const float b0 = -2.0f, b1 = 1.0f, a0 = -1.99599f, a1 = 0.99600f;
  const float scalar = 32767.0f;
  float sum = 0, chk = 0;
  double m1d = 0.0, bx1 = 0.0;
  const long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; it++) {
    // opaque per iteration: the samples' scaling and conversions stay inside
    // the loop, as in the kernel (where every sample is new)
#pragma unroll
    for (int i = 0; i < kReg; i++) asm volatile("" : "+v"(x[i]));
#pragma unroll
    for (int i = 0; i < kReg; i++) {
#pragma unroll
      for (int c = 0; c < NC; c++) {
        const float v = x[(i + 5 * c) % kReg];
        const float xi = v * scalar;
        const float yi = xi + mem0[c];
        const double yd = (double)yi;
        if (MODE == 4) {
          // the same values: (double)mem1 and b1*x of this sample were formed
          // as soon as they were known (the compiler may do this itself)
          mem0[c] = (float)(m1d + __builtin_fma(-(double)a0, yd, b0 * (double)xi));
          mem1[c] = (float)__builtin_fma(-(double)a1, yd, b1 * (double)xi);
          m1d = (double)mem1[c];
          (void)bx1;
        } else {
          mem0[c] = (float)((double)mem1[c] + __builtin_fma(-(double)a0, yd, b0 * (double)xi));
          mem1[c] = (float)__builtin_fma(-(double)a1, yd, b1 * (double)xi);
        }
        if (MODE == 1 || MODE == 4) {
          sum += v * v;
          chk += yi;
        }
      }
    }
  }
  const long long t1 = __builtin_readcyclecounter();
  float r = sum + chk;
#pragma unroll
  for (int c = 0; c < NC; c++) r += mem0[c] + mem1[c];
  out[gid] = r;
  if (gid == 0) *cyc = t1 - t0;
}

template <int MODE>
void run(const float *in, float *out, long long *cyc, int waves_per_simd) {
  const int iters = 256;
  const int nt = 256 * waves_per_simd;
  hipLaunchKernelGGL(kb<MODE>, dim3(256), dim3(nt), 0, 0, in, out, iters, cyc);  // warm
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(kb<MODE>, dim3(256), dim3(nt), 0, 0, in, out, iters, cyc);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  long long c = 0;
  hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  const int nc = MODE == 2 ? 2 : MODE == 3 ? 4 : 1;
  const double samples = (double)iters * kReg;  // per chain
  printf("mode %d  waves/SIMD %d  chains/lane %d  cycles/sample/chain %.1f  cycles/sample/lane %.1f  "
         "(wall %.3f ms; %.2f GHz implied)\n",
         MODE, waves_per_simd, nc, (double)c / (samples * nc), (double)c / samples, ms,
         (double)c / (ms * 1e-3) / 1e9);
}

int main() {
  float *in, *out;
  long long *cyc;
  hipMalloc(&in, 4096 * 4);
  hipMalloc(&out, 256 * 512 * 4);
  hipMalloc(&cyc, 8);
  float h[4096];
  unsigned s = 12345;
  for (int i = 0; i < 4096; i++) {
    s = s * 1664525u + 1013904223u;
    h[i] = ((int)(s >> 9) - (1 << 22)) * (1.0f / (1 << 23));
  }
  hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
  for (int w : {1, 2}) {
    run<0>(in, out, cyc, w);
    run<1>(in, out, cyc, w);
    run<4>(in, out, cyc, w);
    run<2>(in, out, cyc, w);
    run<3>(in, out, cyc, w);
  }
  return 0;
}
