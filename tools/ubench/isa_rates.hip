// Instruction-rate microbenchmark for the VALU ops the stencil kernels use
// (gfx950).  Each kernel runs 8 independent dependency chains per lane so the
// measurement is throughput, not latency.  Prints ns per wave-instruction per
// SIMD equivalent (lower is better) for a full-chip grid.
//
// build: hipcc --offload-arch=gfx950 -O3 tools/ubench/isa_rates.hip -o /tmp/isa_rates
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
using u32 = uint32_t;

#define CHECK(x)                                                          \
  do {                                                                    \
    hipError_t e = (x);                                                   \
    if (e != hipSuccess) {                                                \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);     \
      return 1;                                                           \
    }                                                                     \
  } while (0)

constexpr int ITERS = 4096;

template <int OP>
__global__ __launch_bounds__(256) void k(u32* out, u32 seed, u32 two_bits) {
  u32 a[8];
  uint64_t b[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = seed * (threadIdx.x + 7 * i + 1);
#pragma unroll
  for (int i = 0; i < 8; ++i) b[i] = (uint64_t(a[i]) << 32) | a[(i + 1) & 7];
  const u16x2 two = __builtin_bit_cast(u16x2, two_bits);
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if constexpr (OP == 0) {  // v_pk_add_u16
        a[i] = __builtin_bit_cast(u32, __builtin_bit_cast(u16x2, a[i]) + __builtin_bit_cast(u16x2, a[(i + 1) & 7]));
      } else if constexpr (OP == 1) {  // v_pk_mad_u16
        a[i] = __builtin_bit_cast(u32, __builtin_bit_cast(u16x2, a[i]) * two + __builtin_bit_cast(u16x2, a[(i + 3) & 7]));
      } else if constexpr (OP == 2) {  // v_perm_b32
        a[i] = __builtin_amdgcn_perm(a[i], a[(i + 1) & 7], 0x0c050c01u + it);
      } else if constexpr (OP == 3) {  // v_alignbit_b32
        a[i] = __builtin_amdgcn_alignbit(a[i], a[(i + 1) & 7], 16);
      } else if constexpr (OP == 4) {  // v_mov_b32_dpp wave_shr:1
        a[i] = __builtin_amdgcn_mov_dpp(a[i], 0x138, 0xf, 0xf, true) + 1;
      } else if constexpr (OP == 5) {  // v_mov_b32_dpp row_shr:1
        a[i] = __builtin_amdgcn_mov_dpp(a[i], 0x111, 0xf, 0xf, true) + 1;
      } else if constexpr (OP == 6) {  // v_add_u32 (reference full-rate op)
        a[i] = a[i] + a[(i + 1) & 7];
      } else if constexpr (OP == 7) {  // v_pk_lshrrev_b16
        a[i] = __builtin_bit_cast(u32, __builtin_bit_cast(u16x2, a[i]) >> (u16x2){1, 1}) ^ a[(i + 2) & 7];
      } else if constexpr (OP == 8) {  // ds_swizzle (quad/row perm, LDS crossbar, no memory)
        a[i] = __builtin_amdgcn_ds_swizzle(a[i], 0x041F) + 1;
      } else if constexpr (OP == 9) {  // v_permlane32_swap-free alternative: __shfl_up via ds_bpermute
        a[i] = __shfl_up(a[i], 1) + 1;
      } else if constexpr (OP == 10) {  // v_lshl_add_u64 (shift 0): 64-bit add, four 16-bit SWAR fields
        b[i] = b[i] + b[(i + 1) & 7];
      } else if constexpr (OP == 11) {  // v_lshl_add_u64 (shift 1): b + 2c
        b[i] = (b[(i + 3) & 7] << 1) + b[i];
      } else if constexpr (OP == 12) {  // v_lshrrev_b64
        b[i] = (b[i] >> 4) ^ b[(i + 2) & 7];
      } else if constexpr (OP == 13) {  // v_add3_u32
        a[i] = a[i] + a[(i + 1) & 7] + a[(i + 5) & 7];
      }
    }
  }
  u32 s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s ^= a[i] ^ u32(b[i]) ^ u32(b[i] >> 32);
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int OP>
int run(const char* name, int blocks_per_cu) {
  const int blocks = 256 * blocks_per_cu;
  u32* out;
  CHECK(hipMalloc(&out, blocks * 256 * 4));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  k<OP><<<blocks, 256>>>(out, 3, 0x00020002u);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  k<OP><<<blocks, 256>>>(out, 5, 0x00020002u);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  // wave-instructions of the op: waves * ITERS * 8 ; per SIMD (1024 SIMDs)
  const double waves = blocks * 4.0;
  const double winst = waves * ITERS * 8.0;
  const double per_simd = winst / 1024.0;
  const double cycles = ms * 1e-3 * 2.4e9;
  printf("%-22s blocks/CU=%d  %.3f ms  %.2f cycles per wave-instr per SIMD (at 2.4 GHz)\n", name, blocks_per_cu, ms,
         cycles / per_simd);
  CHECK(hipFree(out));
  return 0;
}

int main() {
  for (int b : {1, 2, 4}) {
    run<6>("v_add_u32", b);
    run<0>("v_pk_add_u16", b);
    run<1>("v_pk_mad_u16", b);
    run<7>("v_pk_lshrrev_b16", b);
    run<2>("v_perm_b32", b);
    run<3>("v_alignbit_b32", b);
    run<4>("dpp wave_shr:1 (+add)", b);
    run<5>("dpp row_shr:1 (+add)", b);
    run<8>("ds_swizzle (+add)", b);
    run<9>("shfl_up/bpermute(+add)", b);
    run<10>("v_lshl_add_u64 (add)", b);
    run<11>("v_lshl_add_u64 (<<1)", b);
    run<12>("v_lshrrev_b64 (+xor)", b);
    run<13>("v_add3_u32", b);
  }
  return 0;
}
