// Microbenchmark (diagnostic): the single-wave level loop of k_chains_glob's
// windowed sweep on synthetic window data (levels of ~25 nodes, 3 in-ring
// links each), with the workgroup's other waves parked at a barrier.
#include <hip/hip_runtime.h>
#include <stdio.h>
#define RING 8192u
#define WN 2048u
#define E 8192u
struct Lds {
  int rv[RING];
  unsigned lev[WN];
  unsigned short aoff[WN], acnt[WN];
  unsigned short adj[E];
  int init[WN];
};
template <int MODE>
__global__ void k(unsigned long long *out, int reps, int per_level) {
  __shared__ Lds L;
  const unsigned tid = threadIdx.x, lane = tid & 63;
  for (unsigned i = tid; i < RING; i += blockDim.x) L.rv[i] = i & 7;
  for (unsigned k = tid; k < WN; k += blockDim.x) {
    L.lev[k] = k / per_level;
    L.aoff[k] = (unsigned short)(3 * k);
    L.acnt[k] = 3;
    L.init[k] = 0;
    for (int t = 0; t < 3; t++) L.adj[(3 * k + t) % E] = (unsigned short)((k * 7 + t * 131) & (RING - 1));
  }
  __syncthreads();
  unsigned long long t0, t1, iters = 0;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  if (tid < 64) {
    for (int r = 0; r < reps; r++) {
      unsigned k = 0;
      const unsigned base = r * 64;
      while (k < WN) {
        const unsigned q = k + lane, kk = q;
        const bool in = q < WN;
        const unsigned lv = in ? L.lev[kk] : 0xFFFFFFFFu;
        const unsigned l = __builtin_amdgcn_readfirstlane(lv);
        const bool mine = in && lv == l;
        const unsigned long long m = __ballot(mine);
        if (mine) {
          const unsigned ao = L.aoff[kk], ac = L.acnt[kk];
          int d = L.init[kk];
          if (MODE == 0) {
            for (unsigned t = 0; t < ac; t++) d = max(d, L.rv[(base + L.adj[ao + t]) & (RING - 1)] + 1);
          }
          L.rv[(base + 4096 + kk) & (RING - 1)] = d;
        }
        k += (unsigned)__popcll(m);
        iters++;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
    }
  }
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  __syncthreads();
  if (tid == 0) {
    out[2 * blockIdx.x] = t1 - t0;
    out[2 * blockIdx.x + 1] = iters;
  }
}
int main() {
  unsigned long long *d, h[2 * 256];
  (void)hipMalloc(&d, sizeof(h));
  for (int mode = 0; mode < 2; mode++)
    for (int bs : {64, 1024})
      for (int pl : {25, 64}) {
        if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(8), dim3(bs), 0, 0, d, 20, pl);
        else hipLaunchKernelGGL(k<1>, dim3(8), dim3(bs), 0, 0, d, 20, pl);
        (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
        printf("mode %d block %d nodes/level %d: ticks/iter %.1f (iters %llu)\n", mode, bs, pl, (double)h[0] / h[1], h[1]);
      }
  return 0;
}
