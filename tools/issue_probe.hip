// issue_probe.hip — issue cost of the vector instructions the codec kernels are made of, on gfx950.
// Each kernel runs ITER blocks of 8 independent instructions of one kind (inline asm, 8 register
// chains) in every lane; 8 waves per SIMD hide each chain's latency, so the time is the SIMD's issue
// cost.  Reported: shader cycles (s_memtime ticks) per wave-instruction per SIMD = one wave's
// elapsed ticks / (its instructions x the waves sharing its SIMD).  LDS rows: one ds_write per
// instruction at a lane stride of 16 bytes plus a byte misalignment (the PCD text stores are
// unaligned 12-byte writes).  LDS atomics need natural alignment: a ds_or_b64 at a 4-byte offset
// aborts the queue (HSA_STATUS_ERROR_MEMORY_APERTURE_VIOLATION, profiles/round5/s03), so only
// aligned atomics are probed.
//   hipcc -O3 --offload-arch=gfx950 tools/issue_probe.hip -o tools/issue_probe && tools/issue_probe
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define R8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#define P8(X) X(0, 8) X(1, 9) X(2, 10) X(3, 11) X(4, 12) X(5, 13) X(6, 14) X(7, 15)
#define D8 "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(d4), "+v"(d5), "+v"(d6), "+v"(d7)
#define U8 "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3), "+v"(u4), "+v"(u5), "+v"(u6), "+v"(u7)

// 32-bit chains (u), 64-bit chains (d, as double or uint64 bits)
#define ADD_U32(i) "v_add_u32 %" #i ", %" #i ", 7\n\t"
#define MUL_F32(i) "v_mul_f32 %" #i ", %" #i ", %" #i "\n\t"
#define MULHI_U24(i) "v_mul_hi_u32_u24 %" #i ", %" #i ", %" #i "\n\t"
#define MUL_U24(i) "v_mul_u32_u24 %" #i ", %" #i ", %" #i "\n\t"
#define MAD_I24(i) "v_mad_i32_i24 %" #i ", %" #i ", %" #i ", %" #i "\n\t"
#define MULLO_U32(i) "v_mul_lo_u32 %" #i ", %" #i ", %" #i "\n\t"
#define MULHI_U32(i) "v_mul_hi_u32 %" #i ", %" #i ", %" #i "\n\t"
#define PKMUL_U16(i) "v_pk_mul_lo_u16 %" #i ", %" #i ", %" #i "\n\t"
#define PKMAD_U16(i) "v_pk_mad_u16 %" #i ", %" #i ", %" #i ", %" #i "\n\t"
#define PERM(i) "v_perm_b32 %" #i ", %" #i ", %" #i ", %" #i "\n\t"
#define ALIGNBIT(i) "v_alignbit_b32 %" #i ", %" #i ", %" #i ", %" #i "\n\t"
#define FFBL(i) "v_ffbl_b32 %" #i ", %" #i "\n\t"
#define BFE(i) "v_bfe_u32 %" #i ", %" #i ", 3, 9\n\t"
#define LSHLOR(i) "v_lshl_or_b32 %" #i ", %" #i ", 4, %" #i "\n\t"
#define ADD3(i) "v_add3_u32 %" #i ", %" #i ", %" #i ", %" #i "\n\t"
#define CVT_F32_U32(i) "v_cvt_f32_u32 %" #i ", %" #i "\n\t"
#define CVT_U32_F32(i) "v_cvt_u32_f32 %" #i ", %" #i "\n\t"
#define RNDNE_F32(i) "v_rndne_f32 %" #i ", %" #i "\n\t"
#define RCP_F32(i) "v_rcp_f32 %" #i ", %" #i "\n\t"
#define MUL_F64(i) "v_mul_f64 %" #i ", %" #i ", %" #i "\n\t"
#define FMA_F64(i) "v_fma_f64 %" #i ", %" #i ", %" #i ", %" #i "\n\t"
#define ADD_F64(i) "v_add_f64 %" #i ", %" #i ", %" #i "\n\t"
#define RNDNE_F64(i) "v_rndne_f64 %" #i ", %" #i "\n\t"
#define FLOOR_F64(i) "v_floor_f64 %" #i ", %" #i "\n\t"
#define LSHR_B64(i) "v_lshrrev_b64 %" #i ", 3, %" #i "\n\t"
#define CVT_F64_F32(i, j) "v_cvt_f64_f32 %" #i ", %" #j "\n\t"
#define CVT_U32_F64(i, j) "v_cvt_u32_f64 %" #j ", %" #i "\n\t"
#define CVT_F64_U32(i, j) "v_cvt_f64_u32 %" #i ", %" #j "\n\t"
#define MAD_U64_U32(i, j) "v_mad_u64_u32 %" #i ", vcc, %" #j ", %" #j ", %" #i "\n\t"

enum Op {
  kAddU32, kMulF32, kMulHiU24, kMulU24, kMadI24, kMulLoU32, kMulHiU32, kPkMulU16, kPkMadU16, kPerm, kAlignbit,
  kFfbl, kBfe, kLshlOr, kAdd3, kCvtF32U32, kCvtU32F32, kRndneF32, kRcpF32, kMulF64, kFmaF64, kAddF64, kRndneF64,
  kFloorF64, kLshrB64, kCvtF64F32, kCvtU32F64, kCvtF64U32, kMadU64U32, kNumOps
};
static const char* kNames[kNumOps] = {
  "v_add_u32", "v_mul_f32", "v_mul_hi_u32_u24", "v_mul_u32_u24", "v_mad_i32_i24", "v_mul_lo_u32", "v_mul_hi_u32",
  "v_pk_mul_lo_u16", "v_pk_mad_u16", "v_perm_b32", "v_alignbit_b32", "v_ffbl_b32", "v_bfe_u32", "v_lshl_or_b32",
  "v_add3_u32", "v_cvt_f32_u32", "v_cvt_u32_f32", "v_rndne_f32", "v_rcp_f32", "v_mul_f64", "v_fma_f64",
  "v_add_f64", "v_rndne_f64", "v_floor_f64", "v_lshrrev_b64", "v_cvt_f64_f32", "v_cvt_u32_f64", "v_cvt_f64_u32",
  "v_mad_u64_u32"};

template <int OP>
__global__ __launch_bounds__(256) void k_valu(uint64_t* out, int iters, uint32_t seed) {
  uint32_t u0 = seed + threadIdx.x, u1 = u0 * 3, u2 = u0 * 5, u3 = u0 * 7, u4 = u0 * 11, u5 = u0 * 13, u6 = u0 * 17,
           u7 = u0 * 19;
  uint64_t d0 = u0 | 0x3ff0000000000000ull, d1 = u1 | 0x3ff0000000000000ull, d2 = u2 | 0x3ff0000000000000ull,
           d3 = u3 | 0x3ff0000000000000ull, d4 = u4 | 0x3ff0000000000000ull, d5 = u5 | 0x3ff0000000000000ull,
           d6 = u6 | 0x3ff0000000000000ull, d7 = u7 | 0x3ff0000000000000ull;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#define U_OP(NAME, M) if constexpr (OP == NAME) asm volatile(R8(M) : U8);
#define D_OP(NAME, M) if constexpr (OP == NAME) asm volatile(R8(M) : D8);
#define DU_OP(NAME, M) if constexpr (OP == NAME) asm volatile(P8(M) : D8, U8 :: "vcc");
    U_OP(kAddU32, ADD_U32) U_OP(kMulF32, MUL_F32) U_OP(kMulHiU24, MULHI_U24) U_OP(kMulU24, MUL_U24)
    U_OP(kMadI24, MAD_I24) U_OP(kMulLoU32, MULLO_U32) U_OP(kMulHiU32, MULHI_U32) U_OP(kPkMulU16, PKMUL_U16)
    U_OP(kPkMadU16, PKMAD_U16) U_OP(kPerm, PERM) U_OP(kAlignbit, ALIGNBIT) U_OP(kFfbl, FFBL) U_OP(kBfe, BFE)
    U_OP(kLshlOr, LSHLOR) U_OP(kAdd3, ADD3) U_OP(kCvtF32U32, CVT_F32_U32) U_OP(kCvtU32F32, CVT_U32_F32)
    U_OP(kRndneF32, RNDNE_F32) U_OP(kRcpF32, RCP_F32)
    D_OP(kMulF64, MUL_F64) D_OP(kFmaF64, FMA_F64) D_OP(kAddF64, ADD_F64) D_OP(kRndneF64, RNDNE_F64)
    D_OP(kFloorF64, FLOOR_F64) D_OP(kLshrB64, LSHR_B64)
    DU_OP(kCvtF64F32, CVT_F64_F32) DU_OP(kCvtU32F64, CVT_U32_F64) DU_OP(kCvtF64U32, CVT_F64_U32)
    DU_OP(kMadU64U32, MAD_U64_U32)
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  const uint64_t sink = (d0 ^ d1 ^ d2 ^ d3 ^ d4 ^ d5 ^ d6 ^ d7) + (u0 ^ u1 ^ u2 ^ u3 ^ u4 ^ u5 ^ u6 ^ u7);
  if ((threadIdx.x & 63) == 0) out[2 * (blockIdx.x * 4 + (threadIdx.x >> 6))] = t1 - t0;
  if (sink == 0x123456789abcdefull) out[1] = sink;   // keeps the chains live
}

// LDS stores: ds_write_bN of each lane at 16 lane + MIS bytes (8 per block, same address)
typedef uint32_t v3u __attribute__((ext_vector_type(3)));
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
#define W1(INS) INS " %0, %1\n\t"
#define W8(INS) W1(INS) W1(INS) W1(INS) W1(INS) W1(INS) W1(INS) W1(INS) W1(INS)
template <int BITS, int MIS>
__global__ __launch_bounds__(256) void k_lds(uint64_t* out, int iters) {
  __shared__ uint4 buf[256 + 2];
  const uint32_t a = (uint32_t)(uintptr_t)(reinterpret_cast<char*>(buf) + 16 * (threadIdx.x & 255) + MIS);
  uint32_t v0 = threadIdx.x;
  const uint64_t w64 = v0 * 3ull;
  const v3u w96 = {v0, v0 + 1, v0 + 2};
  const v4u w128 = {v0, v0 + 1, v0 + 2, v0 + 3};
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    if constexpr (BITS == 8) asm volatile(W8("ds_write_b8") ::"v"(a), "v"(v0) : "memory");
    if constexpr (BITS == 16) asm volatile(W8("ds_write_b16") ::"v"(a), "v"(v0) : "memory");
    if constexpr (BITS == 33) asm volatile(W8("ds_or_b32") ::"v"(a), "v"(v0) : "memory");
    if constexpr (BITS == 65) asm volatile(W8("ds_or_b64") ::"v"(a), "v"(w64) : "memory");
    if constexpr (BITS == 34)
      asm volatile("ds_write2_b32 %0, %1, %1 offset1:1\n\tds_write2_b32 %0, %1, %1 offset1:1\n\t"
                   "ds_write2_b32 %0, %1, %1 offset1:1\n\tds_write2_b32 %0, %1, %1 offset1:1\n\t"
                   "ds_write2_b32 %0, %1, %1 offset1:1\n\tds_write2_b32 %0, %1, %1 offset1:1\n\t"
                   "ds_write2_b32 %0, %1, %1 offset1:1\n\tds_write2_b32 %0, %1, %1 offset1:1\n\t" ::"v"(a), "v"(v0)
                   : "memory");
    if constexpr (BITS == 129) {
      v4u r0, r1;
      asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %2\n\tds_read_b128 %0, %2\n\tds_read_b128 %1, %2\n\t"
                   "ds_read_b128 %0, %2\n\tds_read_b128 %1, %2\n\tds_read_b128 %0, %2\n\tds_read_b128 %1, %2\n\t"
                   "s_waitcnt lgkmcnt(0)"
                   : "=v"(r0), "=v"(r1) : "v"(a) : "memory");
      v0 += r0.x + r1.y;
    }
    if constexpr (BITS == 32) asm volatile(W8("ds_write_b32") ::"v"(a), "v"(v0) : "memory");
    if constexpr (BITS == 64) asm volatile(W8("ds_write_b64") ::"v"(a), "v"(w64) : "memory");
    if constexpr (BITS == 96) asm volatile(W8("ds_write_b96") ::"v"(a), "v"(w96) : "memory");
    if constexpr (BITS == 128) asm volatile(W8("ds_write_b128") ::"v"(a), "v"(w128) : "memory");
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) out[2 * (blockIdx.x * 4 + (threadIdx.x >> 6))] = t1 - t0;
  if (v0 == 0xdeadbeefu) out[1] = v0;
}

template <int BITS, int MIS>
static void run_lds(uint64_t* d_out, uint64_t* h_out, int blocks, int wps, int iters) {
  for (int rep = 0; rep < 2; ++rep) {
    const int n = rep ? iters : 4;
    hipLaunchKernelGGL((k_lds<BITS, MIS>), dim3(blocks), dim3(256), 0, 0, d_out, n);
    if (hipDeviceSynchronize() != hipSuccess) {   // e.g. a misaligned LDS atomic: stop, report nothing more
      fprintf(stderr, "ds %d misaligned %d: kernel failed\n", BITS, MIS);
      exit(3);
    }
    if (!rep) continue;
    hipMemcpy(h_out, d_out, sizeof(uint64_t) * 2 * blocks * 4, hipMemcpyDeviceToHost);
    double sum = 0;
    for (int w = 0; w < blocks * 4; ++w) sum += (double)h_out[2 * w];
    printf("{\"op\": \"ds %d (8/16/32/64/96/128: write_bN, 33: or_b32, 65: or_b64, 34: write2_b32, 129: read_b128) misaligned %d\", \"ticks_per_wave_instr_per_cu\": %.2f}\n", BITS, MIS,
           sum / (blocks * 4) / ((double)n * 8 * wps * 4));
  }
}

template <int OP>
static double run_valu(uint64_t* d_out, uint64_t* h_out, int blocks, int wps, int iters) {
  hipLaunchKernelGGL(k_valu<OP>, dim3(blocks), dim3(256), 0, 0, d_out, iters, 12345u);
  if (hipDeviceSynchronize() != hipSuccess) {
    fprintf(stderr, "%s: kernel failed\n", kNames[OP]);
    exit(3);
  }
  hipMemcpy(h_out, d_out, sizeof(uint64_t) * 2 * blocks * 4, hipMemcpyDeviceToHost);
  double sum = 0;
  for (int w = 0; w < blocks * 4; ++w) sum += (double)h_out[2 * w];
  const double ticks = sum / (blocks * 4);
  return ticks / ((double)iters * 8 * wps);
}

template <int OP>
static void all_ops(uint64_t* d_out, uint64_t* h_out, int blocks, int wps, int iters) {
  if constexpr (OP < kNumOps) {
    run_valu<OP>(d_out, h_out, blocks, wps, 4);   // warm
    const double c = run_valu<OP>(d_out, h_out, blocks, wps, iters);
    printf("{\"op\": \"%s\", \"ticks_per_wave_instr_per_simd\": %.2f}\n", kNames[OP], c);
    all_ops<OP + 1>(d_out, h_out, blocks, wps, iters);
  }
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int wps = 8;                     // waves per SIMD: 8 workgroups of 4 waves per CU
  const int blocks = cus * wps;
  uint64_t* d_out = nullptr;
  if (hipMalloc(&d_out, sizeof(uint64_t) * 2 * blocks * 4) != hipSuccess) return 1;
  static uint64_t h_out[2 * 256 * 8 * 4 * 2];
  if ((size_t)blocks * 8 > sizeof(h_out) / sizeof(h_out[0])) return 1;
  printf("{\"cus\": %d, \"waves_per_simd\": %d}\n", cus, wps);
  all_ops<0>(d_out, h_out, blocks, wps, 2000);
  // LDS: wps workgroups of 4 waves per CU (4 KB each) share the CU's LDS pipe (ticks per wave-instruction per CU)
  run_lds<8, 0>(d_out, h_out, blocks, wps, 500);
  run_lds<8, 1>(d_out, h_out, blocks, wps, 500);
  run_lds<16, 0>(d_out, h_out, blocks, wps, 500);
  run_lds<16, 2>(d_out, h_out, blocks, wps, 500);
  run_lds<33, 0>(d_out, h_out, blocks, wps, 500);
  run_lds<33, 4>(d_out, h_out, blocks, wps, 500);
  run_lds<65, 0>(d_out, h_out, blocks, wps, 500);
  run_lds<34, 0>(d_out, h_out, blocks, wps, 500);
  run_lds<34, 4>(d_out, h_out, blocks, wps, 500);
  run_lds<129, 0>(d_out, h_out, blocks, wps, 500);
  run_lds<129, 4>(d_out, h_out, blocks, wps, 500);
  run_lds<129, 1>(d_out, h_out, blocks, wps, 500);
  run_lds<32, 0>(d_out, h_out, blocks, wps, 500);
  run_lds<64, 0>(d_out, h_out, blocks, wps, 500);
  run_lds<64, 4>(d_out, h_out, blocks, wps, 500);
  run_lds<64, 2>(d_out, h_out, blocks, wps, 500);
  run_lds<96, 0>(d_out, h_out, blocks, wps, 500);
  run_lds<96, 4>(d_out, h_out, blocks, wps, 500);
  run_lds<96, 2>(d_out, h_out, blocks, wps, 500);
  run_lds<96, 1>(d_out, h_out, blocks, wps, 500);
  run_lds<128, 0>(d_out, h_out, blocks, wps, 500);
  run_lds<128, 4>(d_out, h_out, blocks, wps, 500);
  run_lds<128, 1>(d_out, h_out, blocks, wps, 500);
  hipFree(d_out);
  return 0;
}
