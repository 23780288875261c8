// lds_peak.hip — LDS bandwidth CEILINGS on gfx950, measured the way MI355X_MICROARCH.md §LDS
// says its table was measured (VERDICT r04 Weak #2 / item 2): instructions issued continuously,
// no `s_waitcnt lgkmcnt` inside the loop, immediate offsets on one address VGPR (no per-access
// VALU), conflict-free lane-linear addresses.  tools/calib/lds_calib.hip (round 4) computed an
// address and xor-reduced every loaded word (4-5 VALU per ds_read_b64) and drained after each
// group: it measured the VALU and the drain, 0.45-0.49 of the guide's ~150 TB/s for b64 / b128.
//
// Modes (one kernel each, `MODE` template argument):
//   rd64   : 16 x ds_read_b64 per trip                      (guide: 256 B/clk/CU)
//   rd128  :  8 x ds_read_b128 per trip                     (guide: 256 B/clk/CU)
//   wr64   :  8 x ds_write_b64 per trip                     (guide: ~85 B/clk/CU, 6 cycles each)
//   m2s    : the headline kernel's row mix per trip: 15 x ds_read_b64 + 3 x ds_read_b128 +
//            9 x ds_write_b64 (variable phase 7 x (CS gather + V-slot read + v2c store), check
//            phase 3 x b128 + 1 x b64 row reads + CS / argmin-slot stores; bp_reg.h m_var/m_check)
//            = 168 B read + 72 B stored per lane for 224 algorithmic bytes (7 edges x 32 B)
//   m2s8   : config 4's row-of-8 one-word mix (rows of 4 chunks): 16 x b64 + 4 x b128 + 10 x b64
//            stores per lane for 256 algorithmic bytes (8 edges x 32 B)
// Occupancies: the headline's 3 x 256-thread workgroups (52 KiB each) per CU and 4 x 256 (36 KiB).
// The kernel also samples the shader clock (s_memtime against the 100 MHz s_memrealtime) so the
// B/clk/CU figure is measured, not assumed.
//
// Output: one JSON object per (mode, occupancy) on stdout.  Usage on the GPU box:
//   hipcc --offload-arch=gfx950 -O3 -o tools/calib/lds_peak tools/calib/lds_peak.hip && tools/calib/lds_peak
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                            \
  do {                                                                   \
    hipError_t e_ = (x);                                                 \
    if (e_ != hipSuccess) {                                              \
      printf("%s: %s\n", #x, hipGetErrorString(e_));                     \
      return 1;                                                          \
    }                                                                    \
  } while (0)

enum { RD64 = 0, RD128 = 1, WR64 = 2, M2S = 3, M2S8 = 4 };

// one trip of each mode as inline asm; %0 = the lane's byte address (wave segment + lane * 8 or 16)
// and the data registers are dummies (their contents are never consumed: the point is issue rate).
#define R64(off) "ds_read_b64 %1, %0 offset:" #off "\n"
#define R128(off) "ds_read_b128 %2, %0 offset:" #off "\n"
#define W64(off) "ds_write_b64 %0, %3 offset:" #off "\n"

template <int MODE>
__device__ __forceinline__ void trip(uint32_t a64, uint32_t a128) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  uint64_t d64;
  u32x4 d128;
  uint64_t s64 = 0x0123456789abcdefull;
  if (MODE == RD64) {
    asm volatile(R64(0) R64(2048) R64(4096) R64(6144) R64(8192) R64(10240) R64(12288) R64(14336)
                     R64(16384) R64(18432) R64(20480) R64(22528) R64(24576) R64(26624) R64(28672) R64(30720)
                 : "+v"(a64), "=v"(d64), "=v"(d128)
                 : "v"(s64));
  } else if (MODE == RD128) {
    asm volatile(R128(0) R128(4096) R128(8192) R128(12288) R128(16384) R128(20480) R128(24576) R128(28672)
                 : "+v"(a128), "=v"(d64), "=v"(d128)
                 : "v"(s64));
  } else if (MODE == WR64) {
    asm volatile(W64(0) W64(2048) W64(4096) W64(6144) W64(8192) W64(10240) W64(12288) W64(14336)
                 : "+v"(a64), "=v"(d64), "=v"(d128)
                 : "v"(s64));
  } else if (MODE == M2S) {
    // variable phase: per edge a CS gather, a V-slot read and a v2c store (7 edges);
    // check phase: the row (3 x b128 + 1 x b64), then the CS word and the argmin slot
    asm volatile(R64(0) R64(2048) W64(16384) R64(4096) R64(6144) W64(18432) R64(8192) R64(10240) W64(20480)
                     R64(12288) R64(14336) W64(22528) R64(0) R64(2048) W64(24576) R64(4096) R64(6144) W64(26624)
                     R64(8192) R64(10240) W64(28672)
                 : "+v"(a64), "=v"(d64), "=v"(d128)
                 : "v"(s64));
    asm volatile(R128(0) R128(4096) R128(8192) : "+v"(a128), "=v"(d64), "=v"(d128) : "v"(s64));
    asm volatile(R64(12288) W64(30720) W64(32768) : "+v"(a64), "=v"(d64), "=v"(d128) : "v"(s64));
  } else {  // M2S8: 8 edges (16 b64 reads + 8 stores), row of 4 x b128, CS + argmin stores
    asm volatile(R64(0) R64(2048) W64(16384) R64(4096) R64(6144) W64(18432) R64(8192) R64(10240) W64(20480)
                     R64(12288) R64(14336) W64(22528) R64(0) R64(2048) W64(24576) R64(4096) R64(6144) W64(26624)
                     R64(8192) R64(10240) W64(28672) R64(12288) R64(14336) W64(30720)
                 : "+v"(a64), "=v"(d64), "=v"(d128)
                 : "v"(s64));
    asm volatile(R128(0) R128(4096) R128(8192) R128(12288) : "+v"(a128), "=v"(d64), "=v"(d128) : "v"(s64));
    asm volatile(W64(32768) W64(34816) : "+v"(a64), "=v"(d64), "=v"(d128) : "v"(s64));
  }
}

template <int MODE>
__global__ void __launch_bounds__(256) lds_peak(int iters, unsigned long long* clk) {
  extern __shared__ __attribute__((aligned(16))) unsigned char img[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // each wave streams its own 512 B (b64) / 1 KiB (b128) segment inside 2 KiB / 4 KiB strides;
  // stores go to [16 KiB, 36 KiB) (all images are >= 36 KiB)
  const uint32_t base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)img;
  const uint32_t a64 = base + wave * 512 + lane * 8;
  const uint32_t a128 = base + (wave & 3) * 1024 + lane * 16;
  unsigned long long t0 = 0, r0 = 0;
  if (tid == 0) {
    t0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
  }
  for (int it = 0; it < iters; ++it) trip<MODE>(a64, a128);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (tid == 0) {
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (blockIdx.x == 0) {
      clk[0] = t1 - t0;  // shader clocks (vector store)
      clk[1] = r1 - r0;  // 100 MHz ticks
    }
  }
}

struct ModeInfo {
  const char* name;
  double rd_b, wr_b;    // bytes per lane per trip
  double alg_b;         // algorithmic bytes per lane per trip (rows), 0 = not a row mix
  double guide_cycles;  // MI355X_MICROARCH.md §LDS cycles per wave-trip (reads 2 / 4, ds_write_b64 6)
};

template <int MODE>
int run(const ModeInfo& mi, int wg_per_cu, int iters, unsigned long long* clk, int cus) {
  const int img = wg_per_cu == 3 ? 52 * 1024 : 36 * 1024;
  CK(hipFuncSetAttribute((const void*)lds_peak<MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, img));
  const dim3 grid(cus * wg_per_cu), block(256);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL(lds_peak<MODE>, grid, block, img, 0, 16, clk);  // warm-up
  CK(hipEventRecord(a));
  hipLaunchKernelGGL(lds_peak<MODE>, grid, block, img, 0, iters, clk);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  unsigned long long h[2];
  CK(hipMemcpy(h, clk, sizeof(h), hipMemcpyDeviceToHost));
  const double ghz = h[1] ? (double)h[0] / (double)h[1] * 0.1 : 0.0;
  const double lanes = (double)grid.x * 256 * iters, s = ms * 1e-3;
  const double rd = lanes * mi.rd_b, wr = lanes * mi.wr_b;
  // bytes per clock per CU from the in-kernel clock of the first workgroup's wave 0
  const double clocks = (double)h[0];
  const double bpc = clocks > 0 ? (rd + wr) / cus / clocks : 0.0;
  printf("{\"mode\": \"%s\", \"workgroups_per_cu\": %d, \"waves_per_cu\": %d, \"ms\": %.4f, \"TBps\": %.3f, "
         "\"read_TBps\": %.3f, \"write_TBps\": %.3f, \"shader_GHz\": %.4f, \"B_per_clk_per_CU\": %.2f, "
         "\"guide_cycles_per_wave_trip\": %.0f",
         mi.name, wg_per_cu, wg_per_cu * 4, ms, (rd + wr) / s / 1e12, rd / s / 1e12, wr / s / 1e12, ghz, bpc,
         mi.guide_cycles);
  if (mi.alg_b > 0)
    printf(", \"algorithmic_TBps\": %.3f, \"guide_algorithmic_TBps_at_2p4GHz\": %.3f", lanes * mi.alg_b / s / 1e12,
           64.0 * mi.alg_b / mi.guide_cycles * cus * 2.4e9 / 1e12);
  printf("}\n");
  fflush(stdout);
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return 0;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 40000;
  int dev = 0, cus = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  unsigned long long* clk;
  CK(hipMalloc(&clk, 2 * sizeof(unsigned long long)));
  printf("{\"cus\": %d, \"iters\": %d, \"threads\": 256}\n", cus, iters);
  const ModeInfo rd64{"rd64", 16 * 8, 0, 0, 16 * 2}, rd128{"rd128", 8 * 16, 0, 0, 8 * 4},
      wr64{"wr64", 0, 8 * 8, 0, 8 * 6}, m2s{"m2s_row_mix", 15 * 8 + 3 * 16, 9 * 8, 224, 15 * 2 + 3 * 4 + 9 * 6},
      m2s8{"m2s8_row_mix", 16 * 8 + 4 * 16, 10 * 8, 256, 16 * 2 + 4 * 4 + 10 * 6};
  for (int wg : {3, 4}) {
    if (run<RD64>(rd64, wg, iters, clk, cus)) return 1;
    if (run<RD128>(rd128, wg, iters, clk, cus)) return 1;
    if (run<WR64>(wr64, wg, iters, clk, cus)) return 1;
    if (run<M2S>(m2s, wg, iters / 2, clk, cus)) return 1;
    if (run<M2S8>(m2s8, wg, iters / 2, clk, cus)) return 1;
  }
  CK(hipDeviceSynchronize());
  return 0;
}
