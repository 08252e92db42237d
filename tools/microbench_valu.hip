// VALU issue-rate microbenchmark for the SHA-256 kernel's instruction mix on
// gfx950: lane-ops per clock per CU of v_add_u32, v_xor_b32, v_alignbit_b32,
// v_bitop3_b32, v_add3_u32, and the SHA round mix, with 8 independent chains
// per lane and 8 waves per SIMD.  Calibrates the "peak" of the SHA roofline.
// Build: hipcc -O3 --offload-arch=gfx950 tools/microbench_valu.hip -o tools/microbench_valu
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)

constexpr int CH = 8;     // independent chains per lane
constexpr int UNR = 32;   // unrolled steps per loop trip

// inline asm: the compiler cannot fold the chains
template <int OP>
__device__ __forceinline__ uint32_t step(uint32_t x, uint32_t k, uint32_t m) {
  uint32_t r;
  if (OP == 0) asm("v_add_u32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(k));
  if (OP == 1) asm("v_xor_b32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(k));
  if (OP == 2) asm("v_alignbit_b32 %0, %1, %1, 7" : "=v"(r) : "v"(x));
  if (OP == 3) asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(x), "v"(k), "v"(m));
  if (OP == 4) asm("v_add3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(k), "v"(m));
  if (OP == 5) asm("v_perm_b32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(k), "v"(m));
  if (OP == 6) asm("v_alignbyte_b32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(k), "v"(m));
  if (OP == 7) asm("v_bfe_i32 %0, %1, 3, 1" : "=v"(r) : "v"(x));
  if (OP == 8) asm("v_lshl_or_b32 %0, %1, 3, %2" : "=v"(r) : "v"(x), "v"(k));
  if (OP == 9) asm("v_xad_u32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(k), "v"(m));
  if (OP == 10) asm("v_cndmask_b32 %0, %1, %2, vcc" : "=v"(r) : "v"(x), "v"(k));
  if (OP == 11) asm("v_lshrrev_b32 %0, 3, %1" : "=v"(r) : "v"(x));
  // (round 6) the stream kernel's LDS address byte: SDWA byte move into byte 1, rest kept
  if (OP == 12) {
    r = x;  // in place: the chain's own register (no copy)
    asm("v_mov_b32_sdwa %0, %0 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2" : "+v"(r));
  }
  if (OP == 13) asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(k), "v"(m));
  if (OP == 14) asm("v_or_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD" : "=v"(r) : "v"(x), "v"(k));
  if (OP == 15) asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xea" : "=v"(r) : "v"(x), "s"(k), "v"(m));
  if (OP == 16) asm("v_lshlrev_b32_e64 %0, 3, %1" : "=v"(r) : "v"(x));
  if (OP == 17) asm("v_xor_b32_e64 %0, %1, %2" : "=v"(r) : "v"(x), "s"(k));
  if (OP == 18) asm("v_bitop3_b32 %0, %1, 0x3f, %2 bitop3:0xea" : "=v"(r) : "v"(x), "v"(m));
  // selects: the event path's v_cndmask forms against a bitop3 select on a VGPR lane mask
  if (OP == 19) asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(k), "s"((unsigned long long)m * 0x100000001ull));
  if (OP == 20) asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xca" : "=v"(r) : "v"(m), "v"(k), "v"(x));
  if (OP == 21) asm("v_add_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD" : "=v"(r) : "v"(x), "v"(k));
  if (OP == 22) asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(x), "v"(k), "v"(x));
  // SHA-256's forms: the round constant from an SGPR, and a rotate by a 64-bit shift of a register pair
  if (OP == 23) asm("v_add3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "s"(k), "v"(m));
  if (OP == 24) asm("v_add_u32_e32 %0, %1, %2" : "=v"(r) : "s"(k), "v"(x));
  if (OP == 25) {
    uint64_t p = ((uint64_t)x << 32) | m, q;
    asm("v_lshrrev_b64 %0, 13, %1" : "=v"(q) : "v"(p));
    r = (uint32_t)q;
  }
  // the event path's select on VCC: a compare writing VCC, then the select reading it
  if (OP == 26) asm("v_cmp_gt_u32 vcc, %1, %2\n\tv_cndmask_b32 %0, %1, %2, vcc" : "=v"(r) : "v"(x), "v"(k) : "vcc");
  // the same select with the mask in an SGPR pair written by a VOP3 compare
  if (OP == 27) asm("v_cmp_gt_u32_e64 s[100:101], %1, %2\n\tv_cndmask_b32_e64 %0, %1, %2, s[100:101]" : "=v"(r) : "v"(x), "v"(k) : "s100", "s101");
  // a VOP2 op with a literal (non-inline) constant
  if (OP == 28) asm("v_and_b32_e32 %0, 0xff00ff, %1" : "=v"(r) : "v"(x));
  return r;
}

template <int OP>
__global__ __launch_bounds__(512) void k_valu(uint32_t* out, int iters, uint32_t k, uint32_t m) {
  uint32_t c[CH];
#pragma unroll
  for (int i = 0; i < CH; ++i) c[i] = threadIdx.x * 0x9E3779B1u + i;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
#pragma unroll
      for (int i = 0; i < CH; ++i) c[i] = step<OP>(c[i], k + i, m);
    }
  }
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < CH; ++i) r ^= c[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

int main(int argc, char** argv) {
  int iters = argc > 1 ? atoi(argv[1]) : 2000;
  hipDeviceProp_t pr; CK(hipGetDeviceProperties(&pr, 0));
  int ncu = pr.multiProcessorCount;
  int blocks = ncu * 4;  // 4 x 512 threads = 32 waves per CU = 8 per SIMD
  uint32_t* out; CK(hipMalloc(&out, (size_t)blocks * 512 * 4));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const char* names[] = {"v_add_u32", "v_xor_b32", "v_alignbit_b32", "v_bitop3_b32", "v_add3_u32", "v_perm_b32",
                         "v_alignbyte_b32", "v_bfe_i32", "v_lshl_or_b32", "v_xad_u32", "v_cndmask_b32",
                         "v_lshrrev_b32", "v_mov_b32_sdwa", "v_and_or_b32", "v_or_b32_sdwa PAD", "v_bitop3 (s op)", "v_lshlrev_b32_e64", "v_xor_b32_e64 (s)", "v_bitop3 (const)", "v_cndmask_e64 (s mask)", "v_bitop3 select", "v_add_u32_sdwa", "v_bitop3 (x,k,x)", "v_add3_u32 (s op)", "v_add_u32_e32 (s src0)", "v_lshrrev_b64", "v_cmp vcc + v_cndmask_e32", "v_cmp_e64 + v_cndmask_e64", "v_and_b32 literal"};
  const void* fns[] = {(const void*)k_valu<0>, (const void*)k_valu<1>, (const void*)k_valu<2>,
                       (const void*)k_valu<3>, (const void*)k_valu<4>, (const void*)k_valu<5>,
                       (const void*)k_valu<6>, (const void*)k_valu<7>, (const void*)k_valu<8>,
                       (const void*)k_valu<9>, (const void*)k_valu<10>, (const void*)k_valu<11>,
                       (const void*)k_valu<12>, (const void*)k_valu<13>, (const void*)k_valu<14>,
                       (const void*)k_valu<15>, (const void*)k_valu<16>, (const void*)k_valu<17>,
                       (const void*)k_valu<18>, (const void*)k_valu<19>, (const void*)k_valu<20>,
                       (const void*)k_valu<21>, (const void*)k_valu<22>, (const void*)k_valu<23>,
                       (const void*)k_valu<24>, (const void*)k_valu<25>, (const void*)k_valu<26>,
                       (const void*)k_valu<27>, (const void*)k_valu<28>};
  for (int i = 0; i < 29; ++i) {
    uint32_t k = 12345, m = 777;
    void* args[] = {&out, &iters, &k, &m};
    CK(hipLaunchKernel(fns[i], dim3(blocks), dim3(512), args, 0, 0));
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 3; ++r) {
      CK(hipEventRecord(e0));
      CK(hipLaunchKernel(fns[i], dim3(blocks), dim3(512), args, 0, 0));
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best) best = ms;
    }
    double lane_ops = (double)blocks * 512 * iters * UNR * CH;
    printf("%-16s : %8.3f ms  %7.2f T lane-ops/s  %6.1f lane-ops/clk/CU @2.4GHz\n", names[i], best,
           lane_ops / best / 1e9, lane_ops / (best * 1e-3) / ncu / 2.4e9);
  }
  return 0;
}
