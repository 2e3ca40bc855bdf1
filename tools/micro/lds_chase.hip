// Microbenchmark (diagnostic): dependent LDS round trips of one wave, with the
// other waves of the workgroup parked at a barrier; s_memtime vs s_memrealtime.
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k(unsigned long long *out, int iters, int waves_busy) {
  __shared__ unsigned s[8192];
  for (int i = threadIdx.x; i < 8192; i += blockDim.x) s[i] = (i * 97 + 13) & 8191;
  __syncthreads();
  unsigned long long t0, t1, r0, r1;
  unsigned x = threadIdx.x & 63;
  if ((int)(threadIdx.x >> 6) < waves_busy) {
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r0)::"memory");
    for (int i = 0; i < iters; i++) {
      x = s[x];
      __builtin_amdgcn_wave_barrier();
    }
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r1)::"memory");
    if (threadIdx.x == 0) {
      out[3 * blockIdx.x] = t1 - t0;
      out[3 * blockIdx.x + 1] = r1 - r0;
      out[3 * blockIdx.x + 2] = x;
    }
  }
  __syncthreads();
}
int main() {
  unsigned long long *d, h[3 * 256];
  hipMalloc(&d, sizeof(h));
  for (int blocks : {1, 256}) for (int bs : {64, 1024}) {
    int iters = 100000;
    hipLaunchKernelGGL(k, dim3(blocks), dim3(bs), 0, 0, d, iters, 1);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("blocks %d block %d: memtime ticks/iter %.1f  realtime(100MHz) ns/iter %.2f  => clock %.2f GHz\n", blocks, bs,
           (double)h[0] / iters, (double)h[1] * 10.0 / iters, (double)h[0] / (h[1] * 10.0));
  }
  return 0;
}
