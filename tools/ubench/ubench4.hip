// VALU issue-rate microbenchmark (gfx950): cycles per wave-instruction per SIMD for the
// instruction classes the packet kernels are made of. Each thread runs ITERS x 16 independent
// instructions (8 independent chains x 2) in inline asm; the grid fills every SIMD with
// `waves` waves. Rate = total wave-instructions / (SIMDs * kernel cycles).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int ITERS = 4096;

#define OP8(OPS) OPS(v0) OPS(v1) OPS(v2) OPS(v3) OPS(v4) OPS(v5) OPS(v6) OPS(v7)

template <int K>
__global__ __launch_bounds__(256) void k_rate(uint32_t* out, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11, a5 = a0 * 13,
           a6 = a0 * 17, a7 = a0 * 19, b = seed ^ 0x9e3779b9u;
  uint64_t w0 = a0, w1 = a1, w2 = a2, w3 = a3;
  float f0 = a0, f1 = a1, f2 = a2, f3 = a3, f4 = a4, f5 = a5, f6 = a6, f7 = a7, fb = 1.0001f;
  for (int i = 0; i < ITERS; ++i) {
#define R2(I) \
    if (K == 0) asm volatile("v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1" : "+v"(a##I) : "v"(b)); \
    if (K == 1) asm volatile("v_xor_b32 %0, %0, %1\n v_xor_b32 %0, %0, %1" : "+v"(a##I) : "v"(b)); \
    if (K == 2) asm volatile("v_alignbit_b32 %0, %0, %0, 7\n v_alignbit_b32 %0, %0, %0, 7" : "+v"(a##I)); \
    if (K == 3) asm volatile("v_fma_f32 %0, %0, %1, %1\n v_fma_f32 %0, %0, %1, %1" : "+v"(f##I) : "v"(fb)); \
    if (K == 4) asm volatile("v_perm_b32 %0, %0, %1, %1\n v_perm_b32 %0, %0, %1, %1" : "+v"(a##I) : "v"(b)); \
    if (K == 5) asm volatile("v_mul_lo_u32 %0, %0, %1\n v_mul_lo_u32 %0, %0, %1" : "+v"(a##I) : "v"(b)); \
    if (K == 6) asm volatile("v_add3_u32 %0, %0, %1, %1\n v_add3_u32 %0, %0, %1, %1" : "+v"(a##I) : "v"(b)); \
    if (K == 7) asm volatile("v_xad_u32 %0, %0, %1, %1\n v_xad_u32 %0, %0, %1, %1" : "+v"(a##I) : "v"(b)); \
    if (K == 8) asm volatile("v_lshl_or_b32 %0, %0, 3, %1\n v_lshl_or_b32 %0, %0, 3, %1" : "+v"(a##I) : "v"(b)); \
    if (K == 14) asm volatile("v_xor_b32_sdwa %0, %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\n v_xor_b32_sdwa %0, %0, %1 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1" : "+v"(a##I) : "v"(b)); \
    if (K == 15) asm volatile("v_add_u32_e64 %0, %0, %1\n v_add_u32_e64 %0, %0, %1" : "+v"(a##I) : "v"(b)); \
    if (K == 16) asm volatile("v_lshlrev_b32 %0, 3, %0\n v_lshrrev_b32 %0, 3, %0" : "+v"(a##I)); \
    if (K == 17) asm volatile("v_or_b32 %0, %0, %1\n v_and_b32 %0, %0, %1" : "+v"(a##I) : "v"(b)); \
    if (K == 18) asm volatile("v_fmac_f32 %0, %1, %1\n v_fmac_f32 %0, %1, %1" : "+v"(f##I) : "v"(fb)); \
    if (K == 19) asm volatile("v_mul_u32_u24 %0, %0, %1\n v_mul_u32_u24 %0, %0, %1" : "+v"(a##I) : "v"(b)); \
    if (K == 20) asm volatile("v_mov_b32_sdwa %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0\n v_mov_b32_sdwa %0, %1 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1" : "+v"(a##I) : "v"(b)); \
    if (K == 21) asm volatile("v_bfi_b32 %0, %0, %1, %0\n v_bfi_b32 %0, %0, %1, %0" : "+v"(a##I) : "v"(b)); \
    if (K == 22) asm volatile("v_add_co_u32 %0, vcc, %0, %1\n v_addc_co_u32 %0, vcc, %0, %1, vcc" : "+v"(a##I) : "v"(b) : "vcc"); \
    if (K == 27) asm volatile("v_bitop3_b32 %0, %0, %1, %1 bitop3:0x96\n v_bitop3_b32 %0, %0, %1, %1 bitop3:0x96" : "+v"(a##I) : "v"(b)); \
    if (K == 28) asm volatile("v_pk_add_u16 %0, %0, 0 op_sel:[1,0] op_sel_hi:[0,1]\n v_pk_add_u16 %0, %0, 0 op_sel:[1,0] op_sel_hi:[0,1]" : "+v"(a##I)); \
    if (K == 29) asm volatile("v_alignbyte_b32 %0, %0, %0, 2\n v_alignbyte_b32 %0, %0, %0, 2" : "+v"(a##I)); \
    if (K == 31) asm volatile("v_xor_b32_e64 %0, %0, %1\n v_xor_b32_e64 %0, %0, %1" : "+v"(a##I) : "v"(b)); \
    if (K == 32) asm volatile("v_and_or_b32 %0, %0, %1, %1\n v_and_or_b32 %0, %0, %1, %1" : "+v"(a##I) : "v"(b)); \
    if (K == 33) asm volatile("v_xor_b32_dpp %0, %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n v_xor_b32_dpp %0, %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(a##I) : "v"(b)); \
    if (K == 34) asm volatile("v_pk_add_u16 %0, %0, %1\n v_pk_add_u16 %0, %0, %1" : "+v"(a##I) : "v"(b));
    R2(0) R2(1) R2(2) R2(3) R2(4) R2(5) R2(6) R2(7)
    if (K == 9) {  // 64-bit mad: 4 chains x 4
#define M4(I) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0\n v_mad_u64_u32 %0, vcc, %1, %2, %0\n v_mad_u64_u32 %0, vcc, %1, %2, %0\n v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(w##I) : "v"(a0), "v"(b) : "vcc");
      M4(0) M4(1) M4(2) M4(3)
    }
    if (K == 10) {  // packed f32 fma (2 lanes of work per instruction)
      typedef float fv2 __attribute__((ext_vector_type(2)));
      fv2 x0 = {f0, f1}, x1 = {f2, f3}, x2 = {f4, f5}, x3 = {f6, f7}, y = {fb, fb};
#define P4(X) asm volatile("v_pk_fma_f32 %0, %0, %1, %1\n v_pk_fma_f32 %0, %0, %1, %1\n v_pk_fma_f32 %0, %0, %1, %1\n v_pk_fma_f32 %0, %0, %1, %1" : "+v"(X) : "v"(y));
      P4(x0) P4(x1) P4(x2) P4(x3)
      f0 = x0.x; f1 = x0.y; f2 = x1.x; f3 = x1.y; f4 = x2.x; f5 = x2.y; f6 = x3.x; f7 = x3.y;
    }
    if (K == 23) {  // grouped by type across 8 chains: 8 add, 8 xor, 8 alignbit
#define GA(I) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a##I) : "v"(b));
#define GX(I) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a##I) : "v"(b));
#define GR(I) asm volatile("v_alignbit_b32 %0, %0, %0, 16" : "+v"(a##I));
#define G8(M) M(0) M(1) M(2) M(3) M(4) M(5) M(6) M(7)
      G8(GA) G8(GX) G8(GR)
    }
    if (K == 24) {  // add/xor only, grouped
      G8(GA) G8(GX)
    }
    if (K == 25) {  // grouped by 4: 4 add, 4 xor, 4 align (the compiled ChaCha round shape)
      GA(0) GA(1) GA(2) GA(3) GX(0) GX(1) GX(2) GX(3) GR(0) GR(1) GR(2) GR(3)
      GA(4) GA(5) GA(6) GA(7) GX(4) GX(5) GX(6) GX(7) GR(4) GR(5) GR(6) GR(7)
    }
    if (K == 26) {  // fast ops in runs of 16, then 8 slow
      G8(GA) G8(GA) G8(GX) G8(GX) G8(GR) G8(GR)
    }
    if (K == 11) {  // mixed ChaCha-like: add, xor, alignbit
#define Q(I) asm volatile("v_add_u32 %0, %0, %1\n v_xor_b32 %0, %0, %1\n v_alignbit_b32 %0, %0, %0, 16" : "+v"(a##I) : "v"(b));
      Q(0) Q(1) Q(2) Q(3) Q(4) Q(5) Q(6) Q(7)
    }
    if (K == 12) {  // v_mul_hi_u32
#define H2(I) asm volatile("v_mul_hi_u32 %0, %0, %1\n v_mul_hi_u32 %0, %0, %1" : "+v"(a##I) : "v"(b));
      H2(0) H2(1) H2(2) H2(3) H2(4) H2(5) H2(6) H2(7)
    }
    if (K == 13) {  // v_lshlrev_b64 / v_add_co pair (64-bit adds)
#define A4(I) asm volatile("v_lshl_add_u64 %0, %0, 0, %0\n v_lshl_add_u64 %0, %0, 0, %0\n v_lshl_add_u64 %0, %0, 0, %0\n v_lshl_add_u64 %0, %0, 0, %0" : "+v"(w##I));
      A4(0) A4(1) A4(2) A4(3)
    }
  }
  uint32_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ (uint32_t)(w0 ^ w1 ^ w2 ^ w3) ^
               __float_as_uint(f0 + f1 + f2 + f3 + f4 + f5 + f6 + f7);
  if (r == 0x12345678u) out[0] = r;
}

template <int K>
int run(const char* name, int instr_per_iter, int waves_per_simd) {
  uint32_t* out;
  CK(hipMalloc(&out, 4));
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  const int blocks = cus * waves_per_simd;  // 256 threads = 4 waves = one per SIMD
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k_rate<K>, dim3(blocks), dim3(256), 0, 0, out, 1u);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  hipLaunchKernelGGL(k_rate<K>, dim3(blocks), dim3(256), 0, 0, out, 1u);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double clk = p.clockRate * 1e3;  // Hz (max)
  const double wave_instr = (double)blocks * 4 * ITERS * instr_per_iter;
  const double per_simd = wave_instr / (cus * 4.0);
  printf("%-16s waves/SIMD=%d  %.3f ms  %.2f cyc/wave-instr @%.0f MHz  (%.1f G wave-instr/s)\n", name,
         waves_per_simd, ms, (ms * 1e-3 * clk) / per_simd, clk / 1e6, wave_instr / (ms * 1e-3) / 1e9);
  CK(hipFree(out));
  return 0;
}

int main(int argc, char** argv) {
  if (argc > 1) {  // round-2 additions: 3-input / packed / DPP forms
    for (int w : {2, 4, 8}) {
      run<1>("v_xor_b32", 16, w);
      run<31>("v_xor_b32_e64", 16, w);
      run<27>("v_bitop3_b32", 16, w);
      run<28>("v_pk_add_u16 swap", 16, w);
      run<34>("v_pk_add_u16", 16, w);
      run<29>("v_alignbyte_b32", 16, w);
      run<32>("v_and_or_b32", 16, w);
      run<33>("v_xor_b32_dpp", 16, w);
      run<2>("v_alignbit_b32", 16, w);
    }
    return 0;
  }
  for (int w : {2, 4, 8}) {
    run<23>("grp8 add/xor/align", 24, w);
    run<24>("grp8 add/xor", 16, w);
    run<25>("grp4 add/xor/align", 24, w);
    run<26>("grp8 x2", 48, w);
    run<11>("add/xor/align", 24, w);
    run<0>("v_add_u32", 16, w);
    run<2>("v_alignbit_b32", 16, w);
  }
  return 0;
  for (int w : {2, 4}) {
    run<14>("v_xor_b32_sdwa", 16, w);
    run<15>("v_add_u32_e64", 16, w);
    run<16>("v_lshl/lshr_b32", 16, w);
    run<17>("v_or/and_b32", 16, w);
    run<18>("v_fmac_f32", 16, w);
    run<19>("v_mul_u32_u24", 16, w);
    run<20>("v_mov_b32_sdwa", 16, w);
    run<21>("v_bfi_b32", 16, w);
    run<22>("v_add_co/addc", 16, w);
  }
  for (int w : {1, 2, 4}) {
    run<0>("v_add_u32", 16, w);
    run<1>("v_xor_b32", 16, w);
    run<2>("v_alignbit_b32", 16, w);
    run<3>("v_fma_f32", 16, w);
    run<4>("v_perm_b32", 16, w);
    run<5>("v_mul_lo_u32", 16, w);
    run<6>("v_add3_u32", 16, w);
    run<7>("v_xad_u32", 16, w);
    run<8>("v_lshl_or_b32", 16, w);
    run<9>("v_mad_u64_u32", 16, w);
    run<10>("v_pk_fma_f32", 16, w);
    run<11>("add/xor/align", 24, w);
    run<12>("v_mul_hi_u32", 16, w);
    run<13>("v_lshl_add_u64", 16, w);
  }
  return 0;
}
