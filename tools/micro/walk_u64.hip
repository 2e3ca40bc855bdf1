// Microbenchmark (diagnostic): the per-level step of a windowed Kahn-order
// walk with u64 values (64 diff entries per word), one wave, everything in
// LDS.  A step = one level segment of <= 64 positions: its links (four u16
// ring slots packed in a u64, 0xFFFF -> a zero sink slot) and init word were
// loaded one step ahead; the step reads four ring values, ORs, writes its own
// slot.  No ballot, no readfirstlane of a per-node level: segment bounds come
// from a precomputed list.
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/walk_u64 tools/micro/walk_u64.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#define RING 4096u
#define WN 2048u
#define SINK RING
struct Lds {
  unsigned long long ring[RING + 64];
  unsigned long long lk[WN];
  unsigned long long init[WN];
  unsigned seg[WN];
};
template <bool GSTORE>
__global__ __launch_bounds__(256) void k(unsigned long long *out, unsigned long long *gval, int reps, int per_seg,
                                         int nlinks) {
  __shared__ Lds L;
  const unsigned tid = threadIdx.x, lane = tid & 63;
  for (unsigned i = tid; i < RING + 64; i += blockDim.x) L.ring[i] = i < RING ? (1ull << (i & 63)) : 0ull;
  const unsigned nseg = WN / per_seg;
  for (unsigned s = tid; s < WN; s += blockDim.x) L.seg[s] = s < nseg ? ((s * per_seg) | ((unsigned)per_seg << 16)) : 0u;
  for (unsigned q = tid; q < WN; q += blockDim.x) {
    unsigned long long a = 0;
    for (int t = 0; t < 4; t++) {
      const unsigned long long u = t < nlinks ? ((q * 7 + t * 131 + 2048) & (RING - 1)) : SINK;
      a |= u << (16 * t);
    }
    L.lk[q] = a;
    L.init[q] = (q & 1) ? 0ull : (1ull << (q & 63));
  }
  __syncthreads();
  unsigned long long t0, t1, iters = 0;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  if (tid < 64) {
    for (int r = 0; r < reps; r++) {
      const unsigned w0 = (r & 1) * WN;
      unsigned sg = L.seg[0];
      unsigned q = (sg & 0xFFFFu) + lane;
      bool act = lane < (sg >> 16);
      unsigned long long lk = L.lk[act ? q : 0], ini = L.init[act ? q : 0];
      for (unsigned s = 0; s < nseg; s++) {
        const unsigned sg2 = L.seg[s + 1];
        const unsigned q2 = (sg2 & 0xFFFFu) + lane;
        const bool act2 = lane < (sg2 >> 16);
        const unsigned long long lk2 = L.lk[act2 ? q2 : 0], ini2 = L.init[act2 ? q2 : 0];
        const unsigned u0 = (unsigned)lk & 0xFFFFu, u1 = (unsigned)(lk >> 16) & 0xFFFFu,
                       u2 = (unsigned)(lk >> 32) & 0xFFFFu, u3 = (unsigned)(lk >> 48);
        const unsigned long long v = ini | L.ring[u0] | L.ring[u1] | L.ring[u2] | L.ring[u3];
        const unsigned slot = act ? ((w0 + q) & (RING - 1)) : SINK + 1 + lane % 63;
        L.ring[slot] = v;
        if (GSTORE && act) gval[w0 + q] = v;
        iters++;
        q = q2;
        act = act2;
        lk = lk2;
        ini = ini2;
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
  unsigned long long *d, *g, h[2 * 256];
  (void)hipMalloc(&d, sizeof(h));
  (void)hipMalloc(&g, 8 * 2 * WN * 8);
  for (int gs = 0; gs < 2; gs++)
    for (int nl : {1, 4})
      for (int ps : {44, 64}) {
        if (gs)
          hipLaunchKernelGGL(k<true>, dim3(8), dim3(256), 0, 0, d, g, 20, ps, nl);
        else
          hipLaunchKernelGGL(k<false>, dim3(8), dim3(256), 0, 0, d, g, 20, ps, nl);
        hipError_t e = hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
        printf("gstore %d links %d seg %d: ticks/step %.1f (steps %llu) %s\n", gs, nl, ps, (double)h[0] / h[1], h[1],
               hipGetErrorString(e));
      }
  return 0;
}
