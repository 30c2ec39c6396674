// valu_issue_bench.hip -- VALU issue rate of the instruction kinds the scan
// kernel is built from (tuning aid, not product code).
//
// Every lane runs ITER iterations of 16 independent instructions of one kind
// (inline asm, so the exact encoding is issued; DPP operands are read without
// hazard padding -- the values are meaningless, only the timing matters) at
// W waves per SIMD.  Prints wave64-instructions per cycle per SIMD from the
// kernel time (at the nominal 2.4 GHz; the chip may clock lower).
//   hipcc --offload-arch=gfx950 -O3 -o tools/vib tools/valu_issue_bench.hip
//   tools/vib [kind] [waves per SIMD]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#ifndef ITER
#define ITER 4096
#endif

#define X16(S) S(0) S(1) S(2) S(3) S(4) S(5) S(6) S(7) S(8) S(9) S(10) S(11) S(12) S(13) S(14) S(15)

template <int KIND>
__global__ void __launch_bounds__(256) kern(uint32_t* out, uint32_t seed) {
  uint32_t r[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) r[i] = seed * (threadIdx.x + 7u * i + 1u);
  uint32_t b = seed ^ threadIdx.x, c = seed + threadIdx.x;
  // a lane mask in an SGPR pair, written once before the loop (kinds 31-33)
  const uint64_t lm = __builtin_amdgcn_ballot_w64((threadIdx.x & 5) != 0);
  const uint64_t lm2 = __builtin_amdgcn_ballot_w64((threadIdx.x & 6) != 0);
  if constexpr (KIND >= 34) asm volatile("v_cmp_ne_u32 vcc, 0, %0" : : "v"(threadIdx.x & 3) : "vcc");
  for (int it = 0; it < ITER; ++it) {
#define OP(i)                                                                                                 \
  if constexpr (KIND == 0) asm volatile("v_and_b32 %0, %1, %0" : "+v"(r[i]) : "v"(b));                         \
  if constexpr (KIND == 1) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x80" : "+v"(r[i]) : "v"(b), "v"(c)); \
  if constexpr (KIND == 2) asm volatile("v_alignbit_b32 %0, %1, %0, 3" : "+v"(r[i]) : "v"(b));                  \
  if constexpr (KIND == 3)                                                                                    \
    asm volatile("v_mov_b32_dpp %0, %1 wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "=v"(r[i]) : "v"(r[(i + 1) & 15])); \
  if constexpr (KIND == 4)                                                                                    \
    asm volatile("v_add_u32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(r[i])); \
  if constexpr (KIND == 5) asm volatile("v_bcnt_u32_b32 %0, %0, %1" : "+v"(r[i]) : "v"(b));                   \
  if constexpr (KIND == 6) asm volatile("v_lshl_or_b32 %0, %0, 1, %1" : "+v"(r[i]) : "v"(b));                 \
  if constexpr (KIND == 7) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(r[i]) : "v"(b), "v"(c));            \
  if constexpr (KIND == 8) asm volatile("v_bfi_b32 %0, %0, %1, %2" : "+v"(r[i]) : "v"(b), "v"(c));             \
  if constexpr (KIND == 9) asm volatile("v_and_b32 %0, %1, %0\n\tv_alignbit_b32 %0, %1, %0, 3" : "+v"(r[i]) : "v"(b)); \
  if constexpr (KIND == 10) asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(r[i]));                              \
  if constexpr (KIND == 11) asm volatile("v_add_u32 %0, %1, %0" : "+v"(r[i]) : "v"(b));                       \
  if constexpr (KIND == 12) asm volatile("v_or_b32 %0, %1, %0" : "+v"(r[i]) : "v"(b));                        \
  if constexpr (KIND == 13) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(r[i]) : "v"(b));              \
  if constexpr (KIND == 14) asm volatile("v_lshlrev_b64 %0, 3, %0" : "+v"(*(uint64_t*)&r[i & 14]));           \
  if constexpr (KIND == 15) asm volatile("v_or3_b32 %0, %0, %1, %2" : "+v"(r[i]) : "v"(b), "v"(c));           \
  if constexpr (KIND == 16) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(r[i]) : "v"(b), "v"(c));        \
  if constexpr (KIND == 17) asm volatile("v_lshrrev_b32 %0, 5, %0" : "+v"(r[i]));                             \
  if constexpr (KIND == 18) asm volatile("v_alignbyte_b32 %0, %1, %0, 1" : "+v"(r[i]) : "v"(b));              \
  if constexpr (KIND == 19) asm volatile("v_and_b32 %0, %1, %0\n\tv_and_b32 %0, %2, %0\n\tv_alignbit_b32 %0, %1, %0, 3" : "+v"(r[i]) : "v"(b), "v"(c)); \
  if constexpr (KIND == 20) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(r[i]) : "v"(b));                       \
  if constexpr (KIND == 21) asm volatile("v_not_b32 %0, %0" : "+v"(r[i]));                                  \
  if constexpr (KIND == 22) asm volatile("v_and_b32 %0, %1, %0\n\tv_xor_b32 %0, %2, %0\n\tv_or_b32 %0, %1, %0" : "+v"(r[i]) : "v"(b), "v"(c)); \
  if constexpr (KIND == 23) asm volatile("v_and_b32 %0, %1, %0\n\tv_xor_b32 %0, %2, %0\n\tv_or_b32 %0, %1, %0\n\tv_alignbit_b32 %0, %1, %0, 3" : "+v"(r[i]) : "v"(b), "v"(c)); \
  if constexpr (KIND == 24) asm volatile("v_and_b32 %0, %1, %0\n\tv_xor_b32 %0, %2, %0\n\tv_or_b32 %0, %1, %0\n\tv_and_b32 %0, %2, %0\n\tv_xor_b32 %0, %1, %0\n\tv_or_b32 %0, %2, %0\n\tv_add_u32 %0, %1, %0\n\tv_alignbit_b32 %0, %1, %0, 3" : "+v"(r[i]) : "v"(b), "v"(c)); \
  if constexpr (KIND == 25) { if ((threadIdx.x >> 6) & 1) asm volatile("v_alignbit_b32 %0, %1, %0, 3" : "+v"(r[i]) : "v"(b)); else asm volatile("v_and_b32 %0, %1, %0" : "+v"(r[i]) : "v"(b)); } \
  if constexpr (KIND == 28) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(r[i]) : "v"(b), "v"(c));            \
  if constexpr (KIND == 29) asm volatile("v_lshrrev_b64 %0, 3, %0" : "+v"(*(uint64_t*)&r[i & 14]));           \
  if constexpr (KIND == 30) asm volatile("v_mov_b32 %0, %1" : "=v"(r[i]) : "v"(r[(i + 3) & 15]));              \
  if constexpr (KIND == 31) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(r[i]) : "v"(b), "s"(lm));   \
  if constexpr (KIND == 32) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2\n\tv_and_b32 %0, %1, %0\n\tv_xor_b32 %0, %3, %0\n\tv_or_b32 %0, %1, %0" : "+v"(r[i]) : "v"(b), "s"(lm), "v"(c)); \
  if constexpr (KIND == 33) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xca\n\tv_and_b32 %0, %1, %0\n\tv_xor_b32 %0, %2, %0\n\tv_or_b32 %0, %1, %0" : "+v"(r[i]) : "v"(b), "v"(c)); \
  if constexpr (KIND == 34) asm volatile("v_cndmask_b32 %0, %0, %1, vcc\n\tv_and_b32 %0, %1, %0\n\tv_xor_b32 %0, %2, %0\n\tv_or_b32 %0, %1, %0" : "+v"(r[i]) : "v"(b), "v"(c)); \
  if constexpr (KIND == 35) asm volatile("v_cndmask_b32_e64 %0, %0, %1, vcc\n\tv_and_b32 %0, %1, %0\n\tv_xor_b32 %0, %2, %0\n\tv_or_b32 %0, %1, %0" : "+v"(r[i]) : "v"(b), "v"(c)); \
  if constexpr (KIND == 36) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %3\n\tv_and_b32 %0, %1, %0\n\tv_xor_b32 %0, %2, %0\n\tv_or_b32 %0, %1, %0" : "+v"(r[i]) : "v"(b), "v"(c), "s"(lm2)); \
  if constexpr (KIND == 37) asm volatile("v_cndmask_b32 %0, %0, %1, vcc\n\tv_cndmask_b32 %0, %0, %2, vcc\n\tv_and_b32 %0, %1, %0\n\tv_xor_b32 %0, %2, %0\n\tv_or_b32 %0, %1, %0" : "+v"(r[i]) : "v"(b), "v"(c)); \
  if constexpr (KIND == 38) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %3\n\tv_cndmask_b32_e64 %0, %0, %2, %3\n\tv_and_b32 %0, %1, %0\n\tv_xor_b32 %0, %2, %0\n\tv_or_b32 %0, %1, %0" : "+v"(r[i]) : "v"(b), "v"(c), "s"(lm2)); \
  if constexpr (KIND == 26) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x80\n\tv_lshrrev_b32 %0, 3, %0" : "+v"(r[i]) : "v"(b), "v"(c));
    X16(OP)
#undef OP
    if constexpr (KIND == 27) {  // KIND 24's instructions, the slow ones clustered: 16 x 7 fast, then 16 alignbit
#define OPF(i) asm volatile("v_and_b32 %0, %1, %0\n\tv_xor_b32 %0, %2, %0\n\tv_or_b32 %0, %1, %0\n\tv_and_b32 %0, %2, %0\n\tv_xor_b32 %0, %1, %0\n\tv_or_b32 %0, %2, %0\n\tv_add_u32 %0, %1, %0" : "+v"(r[i]) : "v"(b), "v"(c));
#define OPS(i) asm volatile("v_alignbit_b32 %0, %1, %0, 3" : "+v"(r[i]) : "v"(b));
      X16(OPF)
      X16(OPS)
#undef OPF
#undef OPS
    }
  }
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc ^= r[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

static const char* kNames[] = {"v_and_b32 (VOP2)",     "v_bitop3_b32 (VOP3)",  "v_alignbit_b32 (VOP3)",
                               "v_mov_b32_dpp wave_shl", "v_add_u32_dpp row_shr", "v_bcnt_u32_b32",
                               "v_lshl_or_b32",        "v_add3_u32",            "v_bfi_b32",
                               "v_and + v_alignbit", "v_lshlrev_b32 (VOP2)", "v_add_u32 (VOP2)",
                               "v_or_b32 (VOP2)", "v_cndmask_b32 (VOP2)", "v_lshlrev_b64", "v_or3_b32",
                               "v_and_or_b32", "v_lshrrev_b32 (VOP2)", "v_alignbyte_b32", "2 v_and + v_alignbit",
                               "v_xor_b32", "v_not_b32 (VOP1)", "3 fast (and xor or)", "3 fast + alignbit",
                               "7 fast + alignbit", "waves: alignbit | and", "bitop3 + lshrrev", "7 fast x16, then alignbit x16",
                               "v_perm_b32", "v_lshrrev_b64", "v_mov_b32", "v_cndmask e64 SGPR-pair mask",
                               "cndmask(s) + 3 fast", "bitop3 select + 3 fast",
                               "cndmask(vcc, e32) + 3 fast", "cndmask(vcc, e64) + 3 fast", "cndmask(s, v_cmp'd) + 3 fast",
                               "2 cndmask(vcc) + 3 fast", "2 cndmask(s) + 3 fast"};

template <int KIND>
static void run(int cus, uint32_t* out, int wps) {
  const int blocks = cus * wps;  // wps blocks of 4 waves per CU = wps waves per SIMD
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  kern<KIND><<<blocks, 256>>>(out, 12345u);  // warm-up
  (void)hipEventRecord(a);
  kern<KIND><<<blocks, 256>>>(out, 12345u);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, a, b);
  const double per = KIND >= 37 ? 5.0 : KIND == 32 || KIND == 33 || KIND >= 34 ? 4.0 : KIND == 9 || KIND == 26 ? 2.0 : (KIND == 19 || KIND == 22 ? 3.0 : (KIND == 23 ? 4.0 : (KIND == 24 || KIND == 27 ? 8.0 : 1.0)));
  const double instr_per_simd = (double)wps * 16.0 * ITER * per;
  const double cyc = ms * 1e-3 * 2.4e9;
  printf("%-24s waves/SIMD %d  %8.3f ms  %.3f wave-instr/cycle/SIMD\n", kNames[KIND], wps, ms, instr_per_simd / cyc);
}

int main(int argc, char** argv) {
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  const int only = argc > 1 ? atoi(argv[1]) : -1;
  const int wps = argc > 2 ? atoi(argv[2]) : 8;
  uint32_t* out;
  (void)hipMalloc(&out, (size_t)cus * 8 * 256 * 4);
#define RUN(k) \
  if (only < 0 || only == k) run<k>(cus, out, wps);
  RUN(0) RUN(1) RUN(2) RUN(3) RUN(4) RUN(5) RUN(6) RUN(7) RUN(8) RUN(9) RUN(10) RUN(11) RUN(12) RUN(13)
  RUN(14) RUN(15) RUN(16) RUN(17) RUN(18) RUN(19) RUN(20) RUN(21) RUN(22) RUN(23) RUN(24) RUN(25) RUN(26) RUN(27)
  RUN(28) RUN(29) RUN(30) RUN(31) RUN(32) RUN(33) RUN(34) RUN(35) RUN(36) RUN(37) RUN(38)
  (void)hipFree(out);
  return 0;
}
