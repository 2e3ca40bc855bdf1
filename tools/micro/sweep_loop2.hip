// Microbenchmark (diagnostic): k_chains_glob's up-sweep loop (fetch-ahead of
// the next batch's node data, eight packed ring links read together, one
// write) on synthetic window data; one wave works, the rest park at a barrier.
#include <hip/hip_runtime.h>
#include <stdio.h>
#define RING 8192u
#define WN 2048u
struct Lds {
  int rv[RING];
  unsigned rc[RING];
  int init[WN];
  unsigned ibc[WN], ibr[WN], lev[WN];
  unsigned long long lk[WN][2];
  unsigned short aoff[WN], acnt[WN], adj[4096];
  unsigned char flg[WN];
  unsigned pad[2000];
};
__global__ void k(unsigned long long *out, int reps, int per_level, int nlinks) {
  __shared__ Lds L;
  const unsigned tid = threadIdx.x, lane = tid & 63;
  const unsigned M = RING - 1;
  for (unsigned i = tid; i < RING; i += blockDim.x) L.rv[i] = i & 7;
  for (unsigned k = tid; k < WN; k += blockDim.x) {
    L.lev[k] = k / per_level;
    unsigned long long a = 0, b = 0;
    for (int t = 0; t < 8; t++) {
      unsigned long long u = t < nlinks ? ((k * 7 + t * 131) & M) : 0xFFFF;
      if (t < 4) a |= u << (16 * t); else b |= u << (16 * (t - 4));
    }
    L.lk[k][0] = a;
    L.lk[k][1] = b;
    L.init[k] = 0;
    L.flg[k] = 0;
  }
  __syncthreads();
  unsigned long long t0, t1, iters = 0;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  if (tid < 64) {
    for (int r = 0; r < reps; r++) {
      const unsigned base = r * 64, w0 = r * 2048, nw = WN;
      unsigned k = 0;
      auto fetch = [&](unsigned k0, unsigned &lv, unsigned long long (&lk)[2], int &ini, unsigned &fl) {
        const unsigned q = k0 + lane;
        const bool in = q < nw;
        const unsigned kc = in ? q : 0u;
        lv = in ? L.lev[kc] : 0xFFFFFFFFu;
        lk[0] = L.lk[kc][0];
        lk[1] = L.lk[kc][1];
        ini = L.init[kc];
        fl = L.flg[kc];
      };
      unsigned lv, fl;
      unsigned long long lk[2];
      int ini;
      fetch(0, lv, lk, ini, fl);
      while (k < nw) {
        const unsigned q = k + lane, kk = q;
        const unsigned l = __builtin_amdgcn_readfirstlane(lv);
        const bool mine = q < nw && lv == l;
        const unsigned long long m = __ballot(mine);
        const unsigned kn = k + (unsigned)__popcll(m);
        unsigned lv2, fl2;
        unsigned long long lk2[2];
        int ini2;
        fetch(kn, lv2, lk2, ini2, fl2);
        if (mine) {
          const unsigned i = w0 + kk;
          unsigned u[8];
#pragma unroll
          for (int h = 0; h < 8; h++) u[h] = (unsigned)(lk[h >> 2] >> (16 * (h & 3))) & 0xFFFFu;
          int d = ini, v[8];
#pragma unroll
          for (int h = 0; h < 8; h++) v[h] = L.rv[(base + u[h]) & M];
          asm volatile("" ::: "memory");
#pragma unroll
          for (int h = 0; h < 8; h++) d = max(d, u[h] != 0xFFFFu ? v[h] + 1 : d);
          if (fl & 2) {
            const unsigned ao = L.aoff[kk], ac = L.acnt[kk];
            for (unsigned t = 8; t < ac; t++) d = max(d, L.rv[(base + L.adj[ao + t - 8]) & M] + 1);
          }
          L.rv[i & M] = d;
        }
        iters++;
        k = kn;
        lv = lv2;
        lk[0] = lk2[0];
        lk[1] = lk2[1];
        ini = ini2;
        fl = fl2;
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
  (void)hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, 0);
  for (int bs : {64, 1024})
    for (int nl : {2, 8}) {
      hipLaunchKernelGGL(k, dim3(8), dim3(bs), 0, 0, d, 20, 25, nl);
      hipError_t e = hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
      printf("block %d links %d: ticks/iter %.1f (iters %llu) %s\n", bs, nl, (double)h[0] / h[1], h[1], hipGetErrorString(e));
    }
  return 0;
}
