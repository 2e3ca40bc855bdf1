// Microbenchmark (diagnostic): one level step of the windowed walk (k_dx.hip
// k_dx_walk), one wave, LDS only, u64 values.  Records of the next step are
// read one step ahead in every mode.
//   mode 0: link-parallel, G groups of 64 links: read the linked values, LDS
//           atomic OR into the owners' slots (k_dx_walk's step)
//   mode 1: position-parallel: each lane owns a position, ORs the values of its
//           (up to 4) linked slots into its own value and writes it (gather)
//   mode 2: as mode 0 with u32 values (ds_or_b32)
//   mode 3: as mode 0 with plain stores instead of atomics (cost reference only)
//   mode 4: as mode 0 with owners in runs of 4 consecutive lanes (rows of 4 links)
//   hipcc -O3 --offload-arch=gfx950 -o tools/micro/bin/walk_step tools/micro/walk_step.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#define RING 4096u
#define NREC 8192u
__global__ __launch_bounds__(256) void k(unsigned long long *out, int mode, int groups, int steps) {
  __shared__ unsigned long long ring[RING + 64];
  __shared__ unsigned rec[NREC];
  __shared__ unsigned long long lk4[2048];
  const unsigned tid = threadIdx.x, lane = tid & 63;
  for (unsigned i = tid; i < RING + 64; i += blockDim.x) ring[i] = 1ull << (i & 63);
  for (unsigned i = tid; i < NREC; i += blockDim.x) {
    const unsigned owner = 64u + (i * 13u) % 2000u, src = (i * 7u + 2048u) & (RING - 1u);
    rec[i] = src | (owner << 16);
  }
  for (unsigned i = tid; i < 2048; i += blockDim.x) {
    unsigned long long a = 0;
    for (int t = 0; t < 4; t++) a |= (unsigned long long)((i * 7 + t * 131 + 2048) & (RING - 1)) << (16 * t);
    lk4[i] = a;
  }
  __syncthreads();
  unsigned long long t0, t1;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  if (tid < 64) {
    if (mode == 2) {
      unsigned *r32 = (unsigned *)ring;
      unsigned rc[4];
      for (int q = 0; q < 4; q++) rc[q] = q < groups ? rec[64 * q + lane] : (RING | ((RING + 1 + lane) << 16));
      for (int s = 0; s < steps; s++) {
        unsigned x[4];
#pragma unroll
        for (int q = 0; q < 4; q++) x[q] = r32[rc[q] & 0xFFFFu];
        unsigned rn[4];
        const unsigned b = ((s + 1) * 256u) & (NREC - 1u);
#pragma unroll
        for (int q = 0; q < 4; q++) rn[q] = q < groups ? rec[b + 64 * q + lane] : (RING | ((RING + 1 + lane) << 16));
#pragma unroll
        for (int q = 0; q < 4; q++) atomicOr(&r32[rc[q] >> 16], x[q]);
#pragma unroll
        for (int q = 0; q < 4; q++) rc[q] = rn[q];
        asm volatile("" ::: "memory");
      }
    } else if (mode == 3 || mode == 4) {
      unsigned rc[4];
      for (int q = 0; q < 4; q++) rc[q] = q < groups ? rec[64 * q + lane] : (RING | ((RING + 1 + lane) << 16));
      for (int s = 0; s < steps; s++) {
        unsigned long long x[4];
#pragma unroll
        for (int q = 0; q < 4; q++) x[q] = ring[rc[q] & 0xFFFFu];
        unsigned rn[4];
        const unsigned b = ((s + 1) * 256u) & (NREC - 1u);
#pragma unroll
        for (int q = 0; q < 4; q++) rn[q] = q < groups ? rec[b + 64 * q + lane] : (RING | ((RING + 1 + lane) << 16));
#pragma unroll
        for (int q = 0; q < 4; q++) {
          if (mode == 3) ring[rc[q] >> 16] = x[q];
          else atomicOr(&ring[64u + ((s * 64u + 16u * q + (lane >> 2)) & 2047u)], x[q]);
        }
#pragma unroll
        for (int q = 0; q < 4; q++) rc[q] = rn[q];
        asm volatile("" ::: "memory");
      }
    } else if (mode == 0) {
      unsigned rc[4];
      for (int q = 0; q < 4; q++) rc[q] = q < groups ? rec[64 * q + lane] : (RING | ((RING + 1 + lane) << 16));
      for (int s = 0; s < steps; s++) {
        unsigned long long x[4];
#pragma unroll
        for (int q = 0; q < 4; q++) x[q] = ring[rc[q] & 0xFFFFu];
        unsigned rn[4];
        const unsigned b = ((s + 1) * 256u) & (NREC - 1u);
#pragma unroll
        for (int q = 0; q < 4; q++) rn[q] = q < groups ? rec[b + 64 * q + lane] : (RING | ((RING + 1 + lane) << 16));
#pragma unroll
        for (int q = 0; q < 4; q++) atomicOr(&ring[rc[q] >> 16], x[q]);
#pragma unroll
        for (int q = 0; q < 4; q++) rc[q] = rn[q];
        asm volatile("" ::: "memory");
      }
    } else {
      unsigned long long l = lk4[lane];
      for (int s = 0; s < steps; s++) {
        const unsigned u0 = (unsigned)l & 0xFFFFu, u1 = (unsigned)(l >> 16) & 0xFFFFu,
                       u2 = (unsigned)(l >> 32) & 0xFFFFu, u3 = (unsigned)(l >> 48);
        const unsigned long long v = ring[u0] | ring[u1] | ring[u2] | ring[u3];
        const unsigned long long ln = lk4[((s + 1) * 64u + lane) & 2047u];
        ring[64u + ((s * 64u + lane) & 2047u)] = v;
        l = ln;
        asm volatile("" ::: "memory");
      }
    }
  }
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  __syncthreads();
  if (tid == 0) out[blockIdx.x] = t1 - t0;
  if (tid < 64 && ring[tid] == 12345) out[1] = 0;  // keep the ring live
}
int main() {
  unsigned long long *d, h[8];
  (void)hipMalloc(&d, sizeof(h));
  const int steps = 20000;
  for (int mode = 0; mode < 5; mode++)
    for (int g = 1; g <= (mode == 1 ? 1 : 4); g += (mode == 1 ? 1 : 3)) {
      hipLaunchKernelGGL(k, dim3(1), dim3(256), 0, 0, d, mode, g, steps);
      hipError_t e = hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
      printf("mode %d groups %d: ticks/step %.1f %s\n", mode, g, (double)h[0] / steps, hipGetErrorString(e));
    }
  return 0;
}
