// lds_calib.hip — achievable LDS bandwidth on gfx950 for the instruction mix of the headline
// kernel (bp_reg.h m2s family, rmc_kernel<double,4,7,11103,4,256,3>), and calibration of
// rocprofv3's SQ_INSTS_LDS_{LOAD,STORE}_BANDWIDTH counters (units of 64 B, "per-simd, emulated").
//
// Per row of 7 edges the m2s kernel moves (VERDICT r03 Weak #2):
//   variable phase: 7 x (ds_read_b64 CS gather + ds_read_b64 V-slot read + ds_write_b64 v2c store)
//   check phase:    3 x ds_read_b128 + 1 x ds_read_b64 (the row: 56 B), 2 x ds_write_b64 (CS, argmin slot)
// = 168 B read (14 b64 + 3 b128 + 1 b64) and 72 B written (9 b64) per row, 240 B of LDS transfer
// for 224 algorithmic bytes (7 edges x 32 B).
//
// Every mode runs the headline's occupancy: 256-thread workgroups, a 52 KiB LDS image each
// (3 workgroups = 12 waves per CU), 3 x 256 workgroups, conflict-free addresses (lane-linear:
// 8 B per lane for b64, 16 B for b128), loads of one row independent of its stores.
//   mode 0 mix     : the row mix above
//   mode 1 rd_mix  : its reads only (14 b64 + 3 b128 + 1 b64)
//   mode 2 wr_mix  : its stores only (9 b64)
//   mode 3 rd64    : 16 x ds_read_b64
//   mode 4 rd128   : 8 x ds_read_b128
//   mix_pipe(2)    : the row mix software-pipelined (1 or 2 rows per loop trip), stores overlapping loads
// Prints per mode: time, LDS bytes moved, TB/s, and for mode 0 the algorithmic-byte equivalent.
// Usage (GPU box): ./lds_calib [iters]   and under  rocprofv3 --pmc SQ_INSTS_LDS_LOAD_BANDWIDTH
// SQ_INSTS_LDS_STORE_BANDWIDTH --kernel-trace -- ./lds_calib  for the counter calibration.
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

typedef __attribute__((address_space(3))) unsigned long long lds_u64;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) u32x4 lds_u128;

constexpr int kThreads = 256;
constexpr int kImage = 52 * 1024;     // the m2s image at n1600: 52.3 KB -> 3 workgroups per CU
constexpr int kReadRegion = 32 * 1024;
constexpr int kWriteBase = 34 * 1024;  // stores into [34 KB, 52 KB)

__device__ __forceinline__ int opaque(int x) {
  asm volatile("" : "+v"(x));
  return x;
}

template <int MODE>
__global__ void __launch_bounds__(kThreads) lds_mix(int iters, unsigned long long* out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char img[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  auto* base = (__attribute__((address_space(3))) unsigned char*)img;  // generic -> LDS address space
  for (int i = tid; i < kImage / 8; i += kThreads) reinterpret_cast<lds_u64*>(base)[i] = (unsigned long long)i * 0x9E37u;
  __syncthreads();
  unsigned long long acc = (unsigned long long)tid;
  // wave segment: 512 B for b64 (64 lanes x 8 B), 1 KiB for b128
  const int o64 = wave * 512 + lane * 8, o128 = wave * 1024 + lane * 16;
  for (int it = 0; it < iters; ++it) {
    const int rot = opaque(it & 7);
    if (MODE == 0 || MODE == 1 || MODE == 3) {
      constexpr int n64 = MODE == 3 ? 16 : 15;  // (16 distinct 2 KiB strides in the 32 KiB read region)  // 14 gathers / slot reads + the row's last 8 B
#pragma unroll
      for (int k = 0; k < n64; ++k) {
        const int off = ((k + rot) * 2048 + o64) & (kReadRegion - 1);
        acc ^= *reinterpret_cast<lds_u64*>(base + off);
      }
    }
    if (MODE == 0 || MODE == 1 || MODE == 4) {
      constexpr int n128 = MODE == 4 ? 8 : 3;  // (8 distinct 4 KiB strides)
#pragma unroll
      for (int k = 0; k < n128; ++k) {
        const int off = ((k + rot) * 4096 + o128) & (kReadRegion - 1);
        const u32x4 v = *reinterpret_cast<lds_u128*>(base + off);
        acc ^= ((unsigned long long)v.x | ((unsigned long long)v.y << 32)) ^ ((unsigned long long)v.z << 7) ^ v.w;
      }
    }
    if (MODE == 0 || MODE == 2) {
      // 9 stores of 8 B per lane: 7 v2c messages, the CS word, the argmin slot
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        const int off = kWriteBase + ((k + rot) % 9) * 2048 + o64;  // 9 x 2 KiB = [34 KB, 52 KB)
        *reinterpret_cast<lds_u64*>(base + off) = acc + (unsigned long long)k;
      }
    }
  }
  if (acc == 0x123456789ull) out[blockIdx.x] = acc;  // keeps the loads
}

// mode 5 "mix_pipe": the row mix software-pipelined like the kernel's variable phase (stores of
// row r issued between the loads of row r + 1, their data from the previous iteration), so the
// read and store paths overlap: 2 loads : 1 store, 15 b64 + 3 b128 loads and 9 b64 stores per row.
template <int ROWS>
__global__ void __launch_bounds__(kThreads) lds_pipe(int iters, unsigned long long* out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char img[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  auto* base = (__attribute__((address_space(3))) unsigned char*)img;
  for (int i = tid; i < kImage / 8; i += kThreads) reinterpret_cast<lds_u64*>(base)[i] = (unsigned long long)i * 0x9E37u;
  __syncthreads();
  const int o64 = wave * 512 + lane * 8, o128 = wave * 1024 + lane * 16;
  unsigned long long prev[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) prev[k] = (unsigned long long)(tid + k);
  unsigned long long acc = 0;
  for (int it = 0; it < iters; ++it) {
    const int rot = opaque(it & 7);
#pragma unroll
    for (int r = 0; r < ROWS; ++r) {
      unsigned long long ld[18];
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        // two loads, then one store of the previous row's data
        const int a = 2 * k, b = 2 * k + 1;
        if (a < 15) {
          ld[a] = *reinterpret_cast<lds_u64*>(base + (((a + rot + r) * 2048 + o64) & (kReadRegion - 1)));
        } else {
          const u32x4 v = *reinterpret_cast<lds_u128*>(base + (((a + rot + r) * 4096 + o128) & (kReadRegion - 1)));
          ld[a] = ((unsigned long long)v.x | ((unsigned long long)v.y << 32)) ^ ((unsigned long long)v.z << 7) ^ v.w;
        }
        if (b < 15) {
          ld[b] = *reinterpret_cast<lds_u64*>(base + (((b + rot + r) * 2048 + o64) & (kReadRegion - 1)));
        } else {
          const u32x4 v = *reinterpret_cast<lds_u128*>(base + (((b + rot + r) * 4096 + o128) & (kReadRegion - 1)));
          ld[b] = ((unsigned long long)v.x | ((unsigned long long)v.y << 32)) ^ ((unsigned long long)v.z << 7) ^ v.w;
        }
        *reinterpret_cast<lds_u64*>(base + kWriteBase + ((k + rot + r) % 9) * 2048 + o64) = prev[k];
      }
#pragma unroll
      for (int k = 0; k < 9; ++k) prev[k] = ld[2 * k] ^ ld[2 * k + 1];
    }
  }
#pragma unroll
  for (int k = 0; k < 9; ++k) acc ^= prev[k];
  if (acc == 0x123456789ull) out[blockIdx.x] = acc;
}

template <int ROWS>
int run_pipe(const char* name, int iters, unsigned long long* out, int cus) {
  const dim3 grid(cus * 3), block(kThreads);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL(lds_pipe<ROWS>, grid, block, kImage, 0, 4, out);
  CK(hipEventRecord(a));
  hipLaunchKernelGGL(lds_pipe<ROWS>, grid, block, kImage, 0, iters, out);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  // per lane and row: 15 x 8 + 3 x 16 = 168 B read, 9 x 8 = 72 B written
  const double rows = (double)grid.x * kThreads * iters * ROWS, s = ms * 1e-3;
  printf("{\"mode\": \"%s\", \"ms\": %.3f, \"read_bytes\": %.6e, \"write_bytes\": %.6e, \"TBps\": %.3f, "
         "\"rows_per_s\": %.6e, \"algorithmic_TBps\": %.3f}\n", name, ms, rows * 168, rows * 72, rows * 240 / s / 1e12,
         rows / s, rows * 224.0 / s / 1e12);
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return 0;
}

template <int MODE>
int run(const char* name, int iters, unsigned long long* out, double rd_b, double wr_b, int cus) {
  const dim3 grid(cus * 3), block(kThreads);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL(lds_mix<MODE>, grid, block, kImage, 0, 4, out);  // warm-up
  CK(hipEventRecord(a));
  hipLaunchKernelGGL(lds_mix<MODE>, grid, block, kImage, 0, iters, out);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  const double lanes = (double)grid.x * kThreads * iters;
  const double rd = lanes * rd_b, wr = lanes * wr_b, s = ms * 1e-3;
  printf("{\"mode\": \"%s\", \"ms\": %.3f, \"read_bytes\": %.6e, \"write_bytes\": %.6e, \"TBps\": %.3f, "
         "\"read_TBps\": %.3f, \"write_TBps\": %.3f", name, ms, rd, wr, (rd + wr) / s / 1e12, rd / s / 1e12,
         wr / s / 1e12);
  if (MODE == 0) {
    // rows of 7 edges per second: 240 B of transfer per row-lane, 224 algorithmic bytes
    const double rows = lanes / 1.0;
    printf(", \"rows_per_s\": %.6e, \"algorithmic_TBps\": %.3f", rows / s, rows * 224.0 / s / 1e12);
  }
  printf("}\n");
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return 0;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 20000;
  int dev = 0, cus = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  unsigned long long* out;
  CK(hipMalloc(&out, sizeof(unsigned long long) * cus * 3));
  CK(hipFuncSetAttribute((const void*)lds_mix<0>, hipFuncAttributeMaxDynamicSharedMemorySize, kImage));
  CK(hipFuncSetAttribute((const void*)lds_mix<1>, hipFuncAttributeMaxDynamicSharedMemorySize, kImage));
  CK(hipFuncSetAttribute((const void*)lds_mix<2>, hipFuncAttributeMaxDynamicSharedMemorySize, kImage));
  CK(hipFuncSetAttribute((const void*)lds_mix<3>, hipFuncAttributeMaxDynamicSharedMemorySize, kImage));
  CK(hipFuncSetAttribute((const void*)lds_mix<4>, hipFuncAttributeMaxDynamicSharedMemorySize, kImage));
  CK(hipFuncSetAttribute((const void*)lds_pipe<1>, hipFuncAttributeMaxDynamicSharedMemorySize, kImage));
  CK(hipFuncSetAttribute((const void*)lds_pipe<2>, hipFuncAttributeMaxDynamicSharedMemorySize, kImage));
  CK(hipFuncSetAttribute((const void*)lds_pipe<4>, hipFuncAttributeMaxDynamicSharedMemorySize, kImage));
  printf("{\"cus\": %d, \"iters\": %d, \"workgroups_per_cu\": 3, \"threads\": %d, \"lds_per_workgroup\": %d}\n", cus,
         iters, kThreads, kImage);
  // bytes per lane per iteration
  if (run<0>("mix", iters, out, 15 * 8 + 3 * 16, 9 * 8, cus)) return 1;
  if (run<1>("rd_mix", iters, out, 15 * 8 + 3 * 16, 0, cus)) return 1;
  if (run<2>("wr_mix", iters, out, 0, 9 * 8, cus)) return 1;
  if (run<3>("rd64", iters, out, 16 * 8, 0, cus)) return 1;
  if (run<4>("rd128", iters, out, 8 * 16, 0, cus)) return 1;
  if (run_pipe<1>("mix_pipe", iters, out, cus)) return 1;
  if (run_pipe<2>("mix_pipe2", iters / 2, out, cus)) return 1;
  if (run_pipe<4>("mix_pipe4", iters / 4, out, cus)) return 1;
  CK(hipDeviceSynchronize());
  return 0;
}
