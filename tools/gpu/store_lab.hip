// Store-pattern lab (round 4): does the order in which a wave writes the 16-B pieces of an NHWC output row matter to the
// HBM write rate?  The 1x1 streaming GEMMs (conv_p1s / conv_p1p) store 16 pixels x 64 B (32 channels) per instruction:
// every 128-B line is written in two halves, and for a K-channel output the two halves of a line come from consecutive
// 32-channel passes, the rest of the pixel row from later passes.  Patterns timed here (bf16 output of M pixels x K):
//   0 full   : lane l of a wave writes bytes [16 l, 16 l + 16) of a 1 KiB contiguous chunk (torch-fill-like)
//   1 halves : the p1s order -- per 32-channel pass, per 16-pixel block: 16 pixels x 64 B
//   2 pairs  : per 64-channel pair of passes: the two 64-B halves of each line by back-to-back instructions
// each with plain or non-temporal (nt) stores.  hipcc --offload-arch=gfx950 -O3 store_lab.hip -o store_lab
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef unsigned u4 __attribute__((ext_vector_type(4)));

template <int PAT, bool NT>
__global__ void __launch_bounds__(256) store_kernel(unsigned short* __restrict__ y, long M, int K, int tiles) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int q = lane >> 4, pl = lane & 15;
  const u4 v = {(unsigned)lane, 1u, 2u, 3u};
  for (int t = blockIdx.x * 4 + wid; t < tiles; t += gridDim.x * 4) {
    const long p0 = (long)t * 64;  // 64 pixels per wave tile
    if (PAT == 0) {
      const long base = p0 * K;  // elements; the tile is 64 * K contiguous elements
      for (int e = lane * 8; e < 64 * K; e += 512) {
        u4* dst = reinterpret_cast<u4*>(y + base + e);
        if (NT) __builtin_nontemporal_store(v, dst);
        else *dst = v;
      }
    } else {
      const int chq = (q & 1) * 16 + (q >> 1) * 8;
      const int step = PAT == 1 ? 32 : 64;
      for (int ct = 0; ct < K; ct += step)
        for (int pb = 0; pb < 4; ++pb)
          for (int h = 0; h < step / 32; ++h) {
            const long m = p0 + pb * 16 + pl;
            u4* dst = reinterpret_cast<u4*>(y + m * K + ct + 32 * h + chq);
            if (NT) __builtin_nontemporal_store(v, dst);
            else *dst = v;
          }
    }
  }
}

template <int PAT, bool NT>
float run(unsigned short* y, long M, int K, int blocks) {
  const int tiles = (int)(M / 64);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  store_kernel<PAT, NT><<<blocks, 256>>>(y, M, K, tiles);
  hipEventRecord(a);
  for (int i = 0; i < 10; ++i) store_kernel<PAT, NT><<<blocks, 256>>>(y, M, K, tiles);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return ms / 10 * 1e3f;
}

int main() {
  const long shapes[][2] = {{32L * 192 * 192, 512}, {32L * 384 * 384, 64}, {32L * 384 * 384, 128}, {32L * 192 * 192, 128}};
  unsigned short* y;
  hipMalloc(&y, 32L * 384 * 384 * 128 * 2 + (1 << 20));
  int dev = 0, cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  for (auto& s : shapes) {
    const long M = s[0];
    const int K = (int)s[1];
    const double gb = 2.0 * M * K / 1e9;
    for (int bpc : {2, 8}) {
      const int blocks = cus * bpc;
      float t0 = run<0, false>(y, M, K, blocks), t1 = run<1, false>(y, M, K, blocks), t2 = run<2, false>(y, M, K, blocks);
      float n0 = run<0, true>(y, M, K, blocks), n1 = run<1, true>(y, M, K, blocks), n2 = run<2, true>(y, M, K, blocks);
      printf("M %ld K %d (%.2f GB) %d blocks/CU: full %.1f us (%.2f TB/s) halves %.1f (%.2f) pairs %.1f (%.2f) | nt: "
             "full %.1f (%.2f) halves %.1f (%.2f) pairs %.1f (%.2f)\n",
             M, K, gb, bpc, t0, gb / t0 * 1e3, t1, gb / t1 * 1e3, t2, gb / t2 * 1e3, n0, gb / n0 * 1e3, n1,
             gb / n1 * 1e3, n2, gb / n2 * 1e3);
    }
  }
  hipFree(y);
  return 0;
}
