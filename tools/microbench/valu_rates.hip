// VALU issue-rate microbenchmark (dev tool, generated then hand-kept): 8 independent chains per lane,
// 1/2/4 waves per SIMD; prints ns per wave-instruction per SIMD.  Build: hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#define N_ITER 32768
template <int OP> __global__ void kern(float* out, uint32_t sv) {
  float a[8]; uint32_t u[8]; float2 p[8]; double dd[8];
  for (int i = 0; i < 8; ++i) { a[i] = threadIdx.x * 1.0f + i; u[i] = threadIdx.x + i; p[i] = make_float2(a[i], a[i] + 1.0f); dd[i] = a[i]; }
  asm volatile("s_mov_b64 vcc, -1\n s_mov_b64 s[20:21], -1" ::: "vcc", "s20", "s21");
  for (int it = 0; it < N_ITER; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if constexpr (OP == 0) asm volatile("v_add_f32 %0, %0, %1" : "+v"(a[i]) : "v"(a[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 1) asm volatile("v_sub_f32 %0, %0, %1" : "+v"(a[i]) : "v"(a[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 2) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a[i]) : "v"(a[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 3) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(a[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 4) asm volatile("v_min_f32 %0, %0, %1" : "+v"(a[i]) : "v"(a[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 5) asm volatile("v_min_f32 %0, %0, |%1|" : "+v"(a[i]) : "v"(a[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 6) asm volatile("v_max_f32 %0, %0, %1" : "+v"(a[i]) : "v"(a[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 7) asm volatile("v_med3_f32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(a[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 8) asm volatile("v_min3_f32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(a[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 9) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(p[i]) : "v"(p[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 10) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(p[i]) : "v"(p[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 11) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(u[i]) : "v"(u[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 12) asm volatile("v_and_b32 %0, %0, %1" : "+v"(u[i]) : "v"(u[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 13) asm volatile("v_or_b32 %0, %0, %1" : "+v"(u[i]) : "v"(u[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 14) asm volatile("v_and_b32 %0, %2, %0" : "+v"(u[i]) : "v"(u[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 15) asm volatile("v_lshlrev_b32 %0, 1, %0" : "+v"(u[i]) : "v"(u[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 16) asm volatile("v_lshrrev_b32 %0, %1, %0" : "+v"(u[i]) : "v"(u[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 17) asm volatile("v_add_u32 %0, %0, %1" : "+v"(u[i]) : "v"(u[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 18) asm volatile("v_add_u32 %0, %2, %0" : "+v"(u[i]) : "v"(u[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 19) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(u[i]) : "v"(u[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 20) asm volatile("v_min_u32 %0, %0, %1" : "+v"(u[i]) : "v"(u[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 21) asm volatile("v_min_i32 %0, %0, %1" : "+v"(u[i]) : "v"(u[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 22) asm volatile("v_mov_b32 %0, %1" : "+v"(u[i]) : "v"(u[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 23) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(u[i]) : "v"(u[(i+1)&7]), "s"(sv) : "vcc", "s20", "s21");
      if constexpr (OP == 24) asm volatile("v_cndmask_b32_e64 %0, %0, %1, s[20:21]" : "+v"(u[i]) : "v"(u[(i+1)&7]), "s"(sv) : "vcc", "s20", "s21");
      if constexpr (OP == 25) asm volatile("v_cmp_eq_f32 vcc, %0, %1" : "+v"(a[i]) : "v"(a[(i+1)&7]), "s"(sv) : "vcc", "s20", "s21");
      if constexpr (OP == 26) asm volatile("v_cmp_eq_f32_e64 s[20:21], %0, %1" : "+v"(a[i]) : "v"(a[(i+1)&7]), "s"(sv) : "vcc", "s20", "s21");
      if constexpr (OP == 27) asm volatile("v_cmp_eq_u32_sdwa vcc, %0, %1 src0_sel:BYTE_3 src1_sel:DWORD" : "+v"(u[i]) : "v"(u[(i+1)&7]), "s"(sv) : "vcc", "s20", "s21");
      if constexpr (OP == 28) asm volatile("v_bitop3_b32 %0, %0, %1, %1 bitop3:0x6c" : "+v"(u[i]) : "v"(u[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 29) asm volatile("v_bitop3_b32 %0, %0, %1, %1 bitop3:0x96" : "+v"(u[i]) : "v"(u[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 30) asm volatile("v_alignbit_b32 %0, %0, %1, 31" : "+v"(u[i]) : "v"(u[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 31) asm volatile("v_lshl_or_b32 %0, %0, 1, %1" : "+v"(u[i]) : "v"(u[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 32) asm volatile("v_and_or_b32 %0, %0, %1, %1" : "+v"(u[i]) : "v"(u[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 33) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(u[i]) : "v"(u[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 34) asm volatile("v_lshl_add_u32 %0, %0, 1, %1" : "+v"(u[i]) : "v"(u[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 35) asm volatile("v_bfi_b32 %0, %0, %1, %1" : "+v"(u[i]) : "v"(u[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 36) asm volatile("v_bfe_u32 %0, %0, 3, 1" : "+v"(u[i]) : "v"(u[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 37) asm volatile("v_perm_b32 %0, %0, %1, %1" : "+v"(u[i]) : "v"(u[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 38) asm volatile("v_max3_f32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(a[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 39) asm volatile("v_cvt_f32_u32 %0, %1" : "+v"(a[i]) : "v"(u[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 40) asm volatile("v_xor_b32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_3" : "+v"(u[i]) : "v"(u[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 41) asm volatile("v_ldexp_f32 %0, %0, %2" : "+v"(a[i]) : "v"(a[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 42) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(p[i]) : "v"(p[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 44) asm volatile("v_ashrrev_i32 %0, 31, %0" : "+v"(u[i]) : "v"(u[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 45) asm volatile("v_addc_co_u32 %0, vcc, %0, %0, vcc" : "+v"(u[i]) : "v"(u[(i+1)&7]), "s"(sv) : "vcc");
      if constexpr (OP == 46) asm volatile("v_mad_u32_u24 %0, %0, %1, %1" : "+v"(u[i]) : "v"(u[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 47) asm volatile("v_sub_f32_e64 %0, |%0|, %1" : "+v"(a[i]) : "v"(a[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 48) asm volatile("v_lshrrev_b32 %0, 5, %0" : "+v"(u[i]) : "v"(u[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 49) asm volatile("v_bfe_i32 %0, %0, 7, 1" : "+v"(u[i]) : "v"(u[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 50) asm volatile("v_cmp_class_f32 vcc, %0, %1" : "+v"(a[i]) : "v"(u[(i+1)&7]), "s"(sv) : "vcc");
      if constexpr (OP == 51) asm volatile("v_min_u32 %0, %0, %1" : "+v"(u[i]) : "v"(u[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 52) asm volatile("v_add_u32 %0, %2, %0" : "+v"(u[i]) : "v"(u[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 53) asm volatile("v_mov_b32 %0, %2" : "+v"(u[i]) : "v"(u[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 54) asm volatile("v_sub_f32 %0, %0, %1 ; sub-abs\n v_max_f32 %0, |%0|, %1" : "+v"(a[i]) : "v"(a[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 55) asm volatile("v_cndmask_b32_e64 %0, %0, %1, vcc" : "+v"(u[i]) : "v"(u[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 56) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(u[i]) : "v"(u[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 57) asm volatile("v_cmp_gt_f32 vcc, %0, %1\n v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[i]) : "v"(a[(i+1)&7]), "s"(sv) : "vcc");
      if constexpr (OP == 58) asm volatile("v_cmp_gt_f32_e64 s[20:21], %0, %1\n v_cndmask_b32_e64 %0, %0, %1, s[20:21]" : "+v"(a[i]) : "v"(a[(i+1)&7]), "s"(sv) : "s20", "s21");
      if constexpr (OP == 59) asm volatile("v_cmp_gt_f32_e64 s[20:21], %0, %1\n v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[i]) : "v"(a[(i+1)&7]), "s"(sv) : "s20", "s21");
      if constexpr (OP == 60) asm volatile("v_add_f64 %0, %0, %1" : "+v"(dd[i]) : "v"(dd[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 61) asm volatile("v_min_f64 %0, %0, %1" : "+v"(dd[i]) : "v"(dd[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 62) asm volatile("v_max_f64 %0, %0, %1" : "+v"(dd[i]) : "v"(dd[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 63) asm volatile("v_cmp_lt_f64 vcc, %0, %1" : "+v"(dd[i]) : "v"(dd[(i+1)&7]), "s"(sv) : "vcc");
      if constexpr (OP == 64) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(dd[i]) : "v"(dd[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 65) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(dd[i]) : "v"(dd[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 66) asm volatile("v_cmp_gt_f64_e64 s[20:21], 0, %0" : "+v"(dd[i]) : "v"(dd[(i+1)&7]), "s"(sv) : "s20", "s21");
      if constexpr (OP == 67) asm volatile("v_add_f64 %0, %0, -%1" : "+v"(dd[i]) : "v"(dd[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 68) asm volatile("v_min_f64 %0, %0, |%1|" : "+v"(dd[i]) : "v"(dd[(i+1)&7]), "s"(sv) );
      if constexpr (OP == 43) asm volatile("v_pk_mov_b32 %0, %0, %1 op_sel:[1,0]" : "+v"(p[i]) : "v"(p[(i+1)&7]), "s"(sv) );
    }
  }
  float r = 0; for (int i = 0; i < 8; ++i) r += a[i] + p[i].x + p[i].y + (float)u[i] + (float)dd[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
template <int OP> void run(const char* name, float* out) {
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1); float ms[3];
  for (int w = 1; w <= 4; w *= 2) { int idx = w == 1 ? 0 : (w == 2 ? 1 : 2);
    kern<OP><<<256, 256 * w>>>(out, 3u); hipEventRecord(e0); kern<OP><<<256, 256 * w>>>(out, 3u); hipEventRecord(e1); hipEventSynchronize(e1);
    hipEventElapsedTime(&ms[idx], e0, e1); }
  double n = (double)N_ITER * 8;
  printf("%-20s ns/instr/SIMD: 1w %.3f  2w %.3f  4w %.3f\n", name, ms[0]*1e6/n, ms[1]*1e6/n/2, ms[2]*1e6/n/4);
}
int main() { float* out; hipMalloc(&out, 256 * 1024 * sizeof(float));
  run<60>("v_add_f64", out);
  run<67>("v_add_f64_neg", out);
  run<61>("v_min_f64", out);
  run<68>("v_min_f64_abs", out);
  run<62>("v_max_f64", out);
  run<63>("v_cmp_lt_f64", out);
  run<66>("v_cmp_gt_f64_e64_0", out);
  run<64>("v_mul_f64", out);
  run<65>("v_fma_f64", out);
  run<0>("v_add_f32", out);
  run<1>("v_sub_f32", out);
  run<2>("v_mul_f32", out);
  run<3>("v_fma_f32", out);
  run<4>("v_min_f32", out);
  run<5>("v_min_f32_abs", out);
  run<6>("v_max_f32", out);
  run<7>("v_med3_f32", out);
  run<8>("v_min3_f32", out);
  run<9>("v_pk_add_f32", out);
  run<10>("v_pk_mul_f32", out);
  run<11>("v_xor_b32", out);
  run<12>("v_and_b32", out);
  run<13>("v_or_b32", out);
  run<14>("v_and_b32_s", out);
  run<15>("v_lshlrev_b32", out);
  run<16>("v_lshrrev_b32", out);
  run<17>("v_add_u32", out);
  run<18>("v_add_u32_s", out);
  run<19>("v_sub_u32", out);
  run<20>("v_min_u32", out);
  run<21>("v_min_i32", out);
  run<22>("v_mov_b32", out);
  run<23>("v_cndmask_vcc", out);
  run<24>("v_cndmask_e64", out);
  run<25>("v_cmp_eq_f32", out);
  run<26>("v_cmp_eq_f32_e64", out);
  run<27>("v_cmp_eq_u32_sdwa", out);
  run<28>("v_bitop3_b32", out);
  run<29>("v_xor3_b32?", out);
  run<30>("v_alignbit_b32", out);
  run<31>("v_lshl_or_b32", out);
  run<32>("v_and_or_b32", out);
  run<33>("v_add3_u32", out);
  run<34>("v_lshl_add_u32", out);
  run<35>("v_bfi_b32", out);
  run<36>("v_bfe_u32", out);
  run<37>("v_perm_b32", out);
  run<38>("v_max3_f32", out);
  run<55>("v_cndmask_e64_vcc", out);
  run<56>("v_cndmask_vcc_noclob", out);
  run<57>("cmp+cndmask_vcc", out);
  run<58>("cmp+cndmask_e64_s", out);
  run<59>("cmp_s+cndmask_vcc", out);
  run<44>("v_ashrrev_i32_c31", out);
  run<45>("v_addc_co_u32_vcc", out);
  run<46>("v_mad_u32_u24", out);
  run<47>("v_sub_f32_abs_e64", out);
  run<48>("v_lshrrev_b32_c5", out);
  run<49>("v_bfe_i32_c", out);
  run<50>("v_cmp_class_f32", out);
  run<51>("v_min_u32_vv", out);
  run<52>("v_add_u32_sv", out);
  run<53>("v_mov_b32_s", out);
  run<39>("v_cvt_f32_u32", out);
  run<40>("v_xor_b32_sdwa", out);
  run<41>("v_ldexp_f32", out);
  run<42>("v_pk_fma_f32", out);
  run<43>("v_pk_mov_b32", out);
  return 0; }
