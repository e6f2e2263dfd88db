// valu_issue_microbench.hip -- VALU issue cost (cycles per wave-instruction per
// SIMD) of the instruction forms the bitsliced AES (tools/bs_aes.h)
// uses, 4 waves per SIMD, 16 independent accumulators, inline asm so the
// compiler cannot fold anything.  Clock from the cycle counter is not used:
// the result is reported at 2.4 GHz and at the s_memtime-measured clock.
// Build: hipcc --offload-arch=gfx950 -O3 tools/valu_issue_microbench.hip -o tools/bsm_valu
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define R16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)

template <int MODE>
__global__ __launch_bounds__(256) void k(int iters, uint32_t s, uint32_t* out, unsigned long long* clk) {
  uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
           a6 = a0 + 6, a7 = a0 + 7, a8 = a0 + 8, a9 = a0 + 9, a10 = a0 + 10, a11 = a0 + 11,
           a12 = a0 + 12, a13 = a0 + 13, a14 = a0 + 14, a15 = a0 + 15;
  uint32_t b = threadIdx.x * 3 + 1, c = threadIdx.x * 5 + 2;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#define OP(i)                                                                                   \
  if (MODE == 0) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a##i) : "v"(b));                   \
  if (MODE == 1) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(a##i) : "s"(s));                   \
  if (MODE == 2) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a##i) : "v"(b), "v"(c)); \
  if (MODE == 3) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a##i) : "v"(b), "s"(s)); \
  if (MODE == 4) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a##i) : "v"(b), "v"(c));       \
  if (MODE == 5) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a##i) : "v"(b), "s"(s));       \
  if (MODE == 6) asm volatile("v_alignbit_b32 %0, %0, %0, 8" : "+v"(a##i));                     \
  if (MODE == 7) asm volatile("v_lshlrev_b32 %0, 4, %0" : "+v"(a##i));                        \
  if (MODE == 8) asm volatile("v_lshlrev_b32 %0, %1, %0" : "+v"(a##i) : "v"(b));               \
  if (MODE == 9) asm volatile("v_alignbit_b32 %0, %0, %0, %1" : "+v"(a##i) : "v"(b));          \
  if (MODE == 10) asm volatile("v_xor_b32 %0, 1, %0" : "+v"(a##i));                            \
  if (MODE == 11) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xe4" : "+v"(a##i) : "v"(b), "v"(c)); \
  if (MODE == 12) asm volatile("v_and_b32 %0, %0, %1" : "+v"(a##i) : "v"(b));                  \
  if (MODE == 13) asm volatile("v_mov_b32 %0, %1" : "=v"(a##i) : "s"(s));                      \
  if (MODE == 14) asm volatile("v_xor_b32_e64 %0, %0, %1" : "+v"(a##i) : "v"(b));              \
  if (MODE == 15) asm volatile("v_bfi_b32 %0, %0, %1, %2" : "+v"(a##i) : "v"(b), "v"(c));      \
  if (MODE == 16) asm volatile("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2" : "+v"(a##i) : "v"(b)); \
  if (MODE == 17) asm volatile("v_or_b32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2 src1_sel:DWORD" : "+v"(a##i) : "v"(b)); \
  if (MODE == 18) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(a##i) : "v"(b), "v"(c));   \
  if (MODE == 19) asm volatile("v_or3_b32 %0, %0, %1, %2" : "+v"(a##i) : "v"(b), "v"(c));      \
  if (MODE == 20) asm volatile("v_lshl_or_b32 %0, %0, 8, %1" : "+v"(a##i) : "v"(b));           \
  if (MODE == 21) asm volatile("v_xor_b32 %0, 0x12345678, %0" : "+v"(a##i));                   \
  if (MODE == 22) asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(a##i));                         \
  if (MODE == 23) asm volatile("v_and_b32 %0, 0xff00, %0" : "+v"(a##i));                       \
  if (MODE == 24) asm volatile("v_mov_b32_dpp %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(a##i) : "v"(b)); \
  if (MODE == 25) asm volatile("v_xor_b32_dpp %0, %1, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(a##i) : "v"(b)); \
  if (MODE == 26) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a##i) : "v"(b));                  \
  if (MODE == 27) asm volatile("v_lshlrev_b32_sdwa %0, %1, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2" : "+v"(a##i) : "v"(b)); \
  if (MODE == 28) asm volatile("v_and_b32_sdwa %0, %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_3 src1_sel:DWORD" : "+v"(a##i) : "v"(b)); \
  if (MODE == 29) asm volatile("v_mov_b32 %0, %1" : "=v"(a##i) : "v"(b));                       \
  if (MODE == 30) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a##i) : "v"(b));          \
  if (MODE == 31) asm volatile("v_lshrrev_b16 %0, 1, %0" : "+v"(a##i));
    R16(OP) R16(OP) R16(OP) R16(OP)
#undef OP
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ a8 ^ a9 ^
                                              a10 ^ a11 ^ a12 ^ a13 ^ a14 ^ a15;
  if (threadIdx.x == 0 && blockIdx.x == 0) *clk = t1 - t0;
}

int main(int argc, char** argv) {
  int cus = 256;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int block = 256, threads = cus * 4 * 64 * 4, iters = 4096;
  uint32_t* d;
  unsigned long long* clk;
  (void)hipMalloc(&d, (size_t)threads * 4);
  (void)hipMalloc(&clk, 8);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const char* names[] = {"v_xor vv", "v_xor sv (VOP2 sgpr)", "bitop3 vvv", "bitop3 vvs",
                         "v_perm vvv", "v_perm vvs", "v_alignbit", "v_lshlrev",
                         "v_lshlrev vv", "v_alignbit vvv", "v_xor inline", "bitop3 0xe4 vvv",
                         "v_and vv", "v_mov s", "v_xor_e64 vv", "v_bfi vvv",
                         "v_mov_sdwa byte1<-byte2 preserve", "v_or_sdwa byte2", "v_and_or vvv",
                         "v_or3 vvv", "v_lshl_or v,8,v", "v_xor literal", "v_bfe_u32 const",
                         "v_and literal", "v_mov_dpp row_shr", "v_xor_dpp quad_perm", "v_add_u32 vv",
                         "v_lshlrev_sdwa byte2", "v_and_sdwa preserve", "v_mov vv", "v_cndmask vcc",
                         "v_lshrrev_b16"};
  int m0 = argc > 1 ? atoi(argv[1]) : 0;
  for (int mode = m0; mode < 32; ++mode) {
    float best = 1e30f;
    unsigned long long cyc = 0;
    for (int rep = 0; rep < 4; ++rep) {
      (void)hipEventRecord(a);
      switch (mode) {
#define L(m) case m: k<m><<<threads / block, block>>>(iters, 0x05010400u, d, clk); break;
        L(0) L(1) L(2) L(3) L(4) L(5) L(6) L(7) L(8) L(9) L(10) L(11) L(12) L(13) L(14) L(15)
        L(16) L(17) L(18) L(19) L(20) L(21) L(22) L(23) L(24) L(25) L(26) L(27) L(28) L(29) L(30) L(31)
#undef L
      }
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      float ms;
      (void)hipEventElapsedTime(&ms, a, b);
      if (rep && ms < best) best = ms;
      (void)hipMemcpy(&cyc, clk, 8, hipMemcpyDeviceToHost);
    }
    const double instr = (double)threads / 64 * iters * 64;  // wave-instructions
    const double per = best * 1e-3 * 2.4e9 * cus * 4 / instr;
    // s_memtime counts shader-clock cycles: one wave's loop = 4 waves/SIMD sharing.
    const double per_memtime = (double)cyc / (iters * 64.0) / 4.0;
    printf("{\"mode\": \"%s\", \"ms\": %.3f, \"cyc_per_wave_instr_at_2p4\": %.2f, "
           "\"cyc_per_wave_instr_memtime\": %.2f}\n", names[mode], best, per, per_memtime);
  }
  return 0;
}
