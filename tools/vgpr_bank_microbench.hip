// vgpr_bank_microbench.hip -- does v_bitop3_b32's issue rate depend on which
// VGPR banks its three sources sit in, and how many waves per SIMD does a
// stream of independent bitop3s need to issue at full rate?  (The
// full-bitslice AES, tools/fbs_aes.h, is 95% bitop3/xor and runs at two waves
// per SIMD.)  Physical registers are fixed in the asm text; 16 independent
// destinations v[64..79] per group, 4 groups per loop trip.
// Build: hipcc --offload-arch=gfx950 -O3 tools/vgpr_bank_microbench.hip -o tools/vbank
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define STR_(x) #x
#define STR(x) STR_(x)

// One instruction per destination d = 64..79.
#define G16(F) F(64) F(65) F(66) F(67) F(68) F(69) F(70) F(71) F(72) F(73) F(74) F(75) F(76) F(77) F(78) F(79)

// P0: sources v1, v2, v3 (banks 1, 2, 3: distinct)
#define P0(d) "v_bitop3_b32 v" STR(d) ", v1, v2, v3 bitop3:0x96\n"
// P1: sources v4, v8, v3 (two in bank 0)
#define P1(d) "v_bitop3_b32 v" STR(d) ", v4, v8, v3 bitop3:0x96\n"
// P2: sources v4, v8, v12 (all bank 0)
#define P2(d) "v_bitop3_b32 v" STR(d) ", v4, v8, v12 bitop3:0x96\n"
// P3: accumulate: d = d ^ v1 ^ v2 (d's bank varies)
#define P3(d) "v_bitop3_b32 v" STR(d) ", v" STR(d) ", v1, v2 bitop3:0x96\n"
// P4: two sources, same bank
#define P4(d) "v_xor_b32 v" STR(d) ", v4, v8\n"
// P5: two sources, different banks
#define P5(d) "v_xor_b32 v" STR(d) ", v4, v5\n"
// P6: dependent pairs: d = d ^ v1 ^ v2, then the next reads the previous d
#define P6(d) "v_bitop3_b32 v" STR(d) ", v" STR(d) ", v1, v2 bitop3:0x96\nv_bitop3_b32 v" STR(d) ", v" STR(d) ", v2, v3 bitop3:0x96\n"

#define CLOB "v1", "v2", "v3", "v4", "v5", "v8", "v12", "v64", "v65", "v66", "v67", "v68", "v69", "v70", \
    "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79"

template <int P>
__global__ __launch_bounds__(256) void k(int iters, uint32_t* out) {
  uint32_t r = 0;
  asm volatile(
      "v_mov_b32 v1, %0\nv_mov_b32 v2, %0\nv_mov_b32 v3, %0\nv_mov_b32 v4, %0\nv_mov_b32 v5, %0\n"
      "v_mov_b32 v8, %0\nv_mov_b32 v12, %0\n" ::"v"(threadIdx.x) : CLOB);
  for (int it = 0; it < iters; ++it) {
    if (P == 0) asm volatile(G16(P0) G16(P0) G16(P0) G16(P0) ::: CLOB);
    if (P == 1) asm volatile(G16(P1) G16(P1) G16(P1) G16(P1) ::: CLOB);
    if (P == 2) asm volatile(G16(P2) G16(P2) G16(P2) G16(P2) ::: CLOB);
    if (P == 3) asm volatile(G16(P3) G16(P3) G16(P3) G16(P3) ::: CLOB);
    if (P == 4) asm volatile(G16(P4) G16(P4) G16(P4) G16(P4) ::: CLOB);
    if (P == 5) asm volatile(G16(P5) G16(P5) G16(P5) G16(P5) ::: CLOB);
    if (P == 6) asm volatile(G16(P6) G16(P6) ::: CLOB);
  }
  asm volatile("v_mov_b32 %0, v64" : "=v"(r)::CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

int main() {
  int cus = 256;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int iters = 4096;
  uint32_t* d;
  (void)hipMalloc(&d, (size_t)cus * 8 * 256 * 4);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const char* names[] = {"bitop3 banks 1,2,3", "bitop3 banks 0,0,3", "bitop3 banks 0,0,0",
                         "bitop3 acc d^=v1^v2", "xor banks 0,0", "xor banks 0,1",
                         "bitop3 dependent pairs"};
  for (int p = 0; p < 7; ++p)
    for (int w : {1, 2, 4}) {
      const int blocks = cus * w;
      float best = 1e30f;
      for (int rep = 0; rep < 4; ++rep) {
        (void)hipEventRecord(a);
        switch (p) {
#define L(m) case m: k<m><<<blocks, 256>>>(iters, d); break;
          L(0) L(1) L(2) L(3) L(4) L(5) L(6)
#undef L
        }
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        if (rep && ms < best) best = ms;
      }
      // wave-instructions per SIMD = waves per SIMD x iters x 64
      const double per_simd = (double)w * iters * 64;
      printf("{\"pattern\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, "
             "\"cyc_per_wave_instr_per_simd_at_2p4\": %.2f}\n",
             names[p], w, best, best * 1e-3 * 2.4e9 / per_simd);
    }
  return 0;
}
