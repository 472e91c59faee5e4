// Issue cost of the exact VALU encodings the SWAR stencil emits (gfx950).
//
// tools/ubench/isa_rates.hip measured intrinsics, so the compiler chose the
// encodings (its "dpp" row is a v_mov_b32_dpp + v_add pair).  Here every
// instruction is spelled out in inline asm: 8 independent registers written
// round-robin (a register is re-read 7 instructions after it was written, past
// every DPP read-after-write hazard), 16 instructions per asm block, ITERS
// blocks per wave.  Reported: cycles per wave-instruction per SIMD at 2.4 GHz
// for 1, 2, 4 and 8 waves per SIMD (256-thread workgroups, 1/2/4/8 per CU).
//
// build: hipcc --offload-arch=gfx950 -O3 tools/ubench/valu_issue.hip -o /tmp/valu_issue
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CHECK(x)                                                      \
  do {                                                                \
    hipError_t e = (x);                                               \
    if (e != hipSuccess) {                                            \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
      return 1;                                                       \
    }                                                                 \
  } while (0)

constexpr int ITERS = 2048;
constexpr int PER_BLOCK = 16;

// One instruction template per op; %0..%7 are the 8 chain registers.
#define R8(T)                                                                     \
  T("%0", "%1", "%2") T("%1", "%2", "%3") T("%2", "%3", "%4") T("%3", "%4", "%5") \
  T("%4", "%5", "%6") T("%5", "%6", "%7") T("%6", "%7", "%0") T("%7", "%0", "%1")

#define I_ADD(d, a, b) "v_add_u32_e32 " d ", " a ", " b "\n"
#define I_ADD_DPP_WSHR(d, a, b) "v_add_u32_dpp " d ", " a ", " b " wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
#define I_ADD_DPP_WSHL(d, a, b) "v_add_u32_dpp " d ", " a ", " b " wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
#define I_ADD_DPP_RSHR(d, a, b) "v_add_u32_dpp " d ", " a ", " b " row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
#define I_MOV_DPP(d, a, b) "v_mov_b32_dpp " d ", " a " wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
#define I_LSHL_ADD(d, a, b) "v_lshl_add_u32 " d ", " a ", 1, " b "\n"
#define I_ADD3(d, a, b) "v_add3_u32 " d ", " a ", " b ", " d "\n"
#define I_LSHR(d, a, b) "v_lshrrev_b32_e32 " d ", 4, " a "\n"
#define I_AND(d, a, b) "v_and_b32_e32 " d ", 0xff00ff, " a "\n"
#define I_PERM(d, a, b) "v_perm_b32 " d ", " a ", " b ", %8\n"
#define I_ADD_LSHL(d, a, b) "v_add_lshl_u32 " d ", " a ", " b ", 1\n"
#define I_BFE(d, a, b) "v_bfe_u32 " d ", " a ", 4, 8\n"
// float ops of the float temporal kernel (stencil_float.hip)
#define I_ADD_F32(d, a, b) "v_add_f32_e32 " d ", " a ", " b "\n"
#define I_MUL_F32(d, a, b) "v_mul_f32_e32 " d ", " a ", " b "\n"
#define I_TRUNC_F32(d, a, b) "v_trunc_f32_e32 " d ", " a "\n"
#define I_CVT_UBYTE(d, a, b) "v_cvt_f32_ubyte1_e32 " d ", " a "\n"
#define I_CVT_PK_U8(d, a, b) "v_cvt_pk_u8_f32 " d ", " a ", 1, " b "\n"
#define I_MED3_F32(d, a, b) "v_med3_f32 " d ", " a ", 0, " b "\n"
// packed f32 on register pairs (%0..%7 are 64-bit operands here)
#define I_PK_ADD_F32(d, a, b) "v_pk_add_f32 " d ", " a ", " b "\n"
#define I_PK_MUL_F32(d, a, b) "v_pk_mul_f32 " d ", " a ", " b "\n"

#define KERNEL(NAME, T)                                                                         \
  __global__ __launch_bounds__(256) void NAME(uint32_t* out, uint32_t seed) {                   \
    uint32_t r0 = seed + threadIdx.x, r1 = r0 * 3, r2 = r0 * 5, r3 = r0 * 7, r4 = r0 * 11,      \
             r5 = r0 * 13, r6 = r0 * 17, r7 = r0 * 19;                                          \
    const uint32_t sel = 0x06020400u + (seed >> 31);                                            \
    for (int it = 0; it < ITERS; ++it) {                                                        \
      asm volatile(R8(T) R8(T)                                                                  \
                   : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7) \
                   : "s"(sel)); \
    }                                                                                           \
    out[blockIdx.x * blockDim.x + threadIdx.x] = r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7;        \
  }

KERNEL(k_add, I_ADD)
KERNEL(k_add_dpp_wshr, I_ADD_DPP_WSHR)
KERNEL(k_add_dpp_wshl, I_ADD_DPP_WSHL)
KERNEL(k_add_dpp_rshr, I_ADD_DPP_RSHR)
KERNEL(k_mov_dpp, I_MOV_DPP)
KERNEL(k_lshl_add, I_LSHL_ADD)
KERNEL(k_add3, I_ADD3)
KERNEL(k_lshr, I_LSHR)
KERNEL(k_and, I_AND)
KERNEL(k_perm, I_PERM)
KERNEL(k_add_lshl, I_ADD_LSHL)
KERNEL(k_bfe, I_BFE)
KERNEL(k_add_f32, I_ADD_F32)
KERNEL(k_mul_f32, I_MUL_F32)
KERNEL(k_trunc_f32, I_TRUNC_F32)
KERNEL(k_cvt_ubyte, I_CVT_UBYTE)
KERNEL(k_cvt_pk_u8, I_CVT_PK_U8)
KERNEL(k_med3_f32, I_MED3_F32)

#define KERNEL64(NAME, T)                                                                       \
  __global__ __launch_bounds__(256) void NAME(uint32_t* out, uint32_t seed) {                   \
    uint64_t r0 = seed + threadIdx.x, r1 = r0 * 3, r2 = r0 * 5, r3 = r0 * 7, r4 = r0 * 11,      \
             r5 = r0 * 13, r6 = r0 * 17, r7 = r0 * 19;                                          \
    for (int it = 0; it < ITERS; ++it) {                                                        \
      asm volatile(R8(T) R8(T)                                                                  \
                   : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7)); \
    }                                                                                           \
    out[blockIdx.x * blockDim.x + threadIdx.x] = uint32_t(r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7); \
  }
KERNEL64(k_pk_add_f32, I_PK_ADD_F32)
KERNEL64(k_pk_mul_f32, I_PK_MUL_F32)

template <typename K>
int run(const char* name, K kern, int per_cu) {
  const int blocks = 256 * per_cu;
  uint32_t* out;
  CHECK(hipMalloc(&out, blocks * 256 * 4));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, 3u);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, 5u);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double winst = blocks * 4.0 * ITERS * PER_BLOCK;  // wave-instructions
  const double cycles = ms * 1e-3 * 2.4e9;
  printf("%-16s waves/SIMD=%d  %.3f ms  %.2f cycles per wave-instr per SIMD\n", name, per_cu, ms,
         cycles / (winst / 1024.0));
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  CHECK(hipFree(out));
  return 0;
}

int main() {
  for (int w : {1, 2, 4, 8}) {
    run("v_add_u32", k_add, w);
    run("add_dpp wave_shr", k_add_dpp_wshr, w);
    run("add_dpp wave_shl", k_add_dpp_wshl, w);
    run("add_dpp row_shr", k_add_dpp_rshr, w);
    run("mov_dpp wave_shr", k_mov_dpp, w);
    run("v_lshl_add_u32", k_lshl_add, w);
    run("v_add3_u32", k_add3, w);
    run("v_lshrrev_b32", k_lshr, w);
    run("v_and_b32 (lit)", k_and, w);
    run("v_perm_b32", k_perm, w);
    run("v_add_lshl_u32", k_add_lshl, w);
    run("v_bfe_u32", k_bfe, w);
    run("v_add_f32", k_add_f32, w);
    run("v_mul_f32", k_mul_f32, w);
    run("v_pk_add_f32", k_pk_add_f32, w);
    run("v_pk_mul_f32", k_pk_mul_f32, w);
    run("v_trunc_f32", k_trunc_f32, w);
    run("v_cvt_f32_ubyte1", k_cvt_ubyte, w);
    run("v_cvt_pk_u8_f32", k_cvt_pk_u8, w);
    run("v_med3_f32", k_med3_f32, w);
  }
  return 0;
}
