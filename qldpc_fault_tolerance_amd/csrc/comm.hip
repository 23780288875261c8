// comm.hip — the multi-GPU half of the C ABI and the standalone
// error sampler.
//
// The shot loop shards by global shot index with no data-path exchange; the one
// collective is a sum of the int64 counter vector (qldpc_counters) per (code, p) --
// the reduction `parmap` + `np.sum` perform over forked workers in the reference
// (src/Simulators.py:37-61, :170-188).  Here it is one RCCL all-reduce over xGMI.
// RCCL is resolved at first use with dlopen (librccl.so.1 of the ROCm install, or
// the copy a host process such as torch already loaded under that soname), so the
// engine library itself carries no link-time dependency on RCCL.
//
// qldpc_sample_errors is the sampling half of the fused kernels on its own
// (src/Simulators.py:89-115 `_generate_error`): the same Philox stream / external
// uniforms and the same 3-way split, for bit-exact sampling parity at the boundary.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <dlfcn.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/qldpc_hip.h"
#include "bp_kernels.h"
#include "runtime.h"

using namespace qldpc_rt;

struct qldpc_comm {
  ncclComm_t comm = nullptr;
  int device = 0, rank = 0, nranks = 1;
};

namespace {

struct Rccl {
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*) = nullptr;
  ncclResult_t (*AllReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  const char* (*GetErrorString)(ncclResult_t) = nullptr;
  bool ok = false;
  std::string why;
};

const Rccl& rccl() {
  static Rccl R;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = nullptr;
    for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
      h = dlopen(name, RTLD_NOW | RTLD_GLOBAL);
      if (h) break;
    }
    if (!h) {
      R.why = std::string("RCCL not loadable (dlopen librccl.so.1): ") + (dlerror() ? dlerror() : "?");
      return;
    }
    bool all = true;
    auto sym = [&](auto& fn, const char* name) {
      fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
      all = all && fn != nullptr;
    };
    sym(R.GetUniqueId, "ncclGetUniqueId");
    sym(R.CommInitRank, "ncclCommInitRank");
    sym(R.CommInitAll, "ncclCommInitAll");
    sym(R.AllReduce, "ncclAllReduce");
    sym(R.GroupStart, "ncclGroupStart");
    sym(R.GroupEnd, "ncclGroupEnd");
    sym(R.CommDestroy, "ncclCommDestroy");
    sym(R.GetErrorString, "ncclGetErrorString");
    R.ok = all;
    if (!all) R.why = "RCCL library lacks an nccl* entry point";
  });
  return R;
}

#define QLDPC_RCCL(x)                                                                                      \
  do {                                                                                                     \
    ncclResult_t r_ = (x);                                                                                 \
    if (r_ != ncclSuccess) return set_err(QLDPC_EHIP, std::string(#x) + ": " + rccl().GetErrorString(r_)); \
  } while (0)

int need_rccl() {
  const Rccl& R = rccl();
  return R.ok ? 0 : set_err(QLDPC_ENOTSUP, R.why);
}

constexpr size_t kCounterWords = sizeof(qldpc_counters) / sizeof(int64_t);

// One thread per (shot, qubit); the class bits as the fused kernels record them in d_err.
__global__ void sample_errors_kernel(unsigned long long seed, unsigned long long shot_begin, long long S, int n,
                                     const double* uniforms, double t1, double t2, double t3, unsigned long long K1,
                                     unsigned long long K2, unsigned long long K3, uint8_t* err) {
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= S * (long long)n) return;
  const long long s = idx / n;
  const int j = (int)(idx - s * n);
  uint32_t cls;
  if (uniforms) {
    const double u = uniforms[idx];
    cls = (u < t1) ? 2u : (t1 <= u && u < t2) ? 1u : (t2 <= u && u < t3) ? 3u : 0u;
  } else {
    const unsigned long long k = qldpc::philox_k53(seed, shot_begin + (unsigned long long)s, (uint32_t)j);
    cls = (k < K1) ? 2u : (k < K2) ? 1u : (k < K3) ? 3u : 0u;
  }
  err[idx] = (uint8_t)cls;
}

unsigned long long ceil53(double t) {
  if (!(t > 0.0)) return 0ull;
  if (t >= 1.0) return 1ull << 53;
  return (unsigned long long)std::ceil(std::ldexp(t, 53));
}

}  // namespace

extern "C" {

int qldpc_comm_unique_id(uint8_t* id_out) {
  if (!id_out) return set_err(QLDPC_EINVAL, "id_out is NULL");
  if (int rc = need_rccl()) return rc;
  ncclUniqueId id;
  QLDPC_RCCL(rccl().GetUniqueId(&id));
  static_assert(sizeof(ncclUniqueId) == QLDPC_COMM_ID_BYTES, "ncclUniqueId size");
  std::memcpy(id_out, &id, sizeof(id));
  return 0;
}

int qldpc_comm_init_rank(int device, int32_t nranks, int32_t rank, const uint8_t* id, qldpc_comm** out) {
  if (!out || !id) return set_err(QLDPC_EINVAL, "NULL argument");
  if (nranks < 1 || rank < 0 || rank >= nranks) return set_err(QLDPC_EINVAL, "rank out of range");
  if (int rc = need_rccl()) return rc;
  QLDPC_HIP(hipSetDevice(device));
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof(uid));
  auto* c = new qldpc_comm();
  c->device = device;
  c->rank = rank;
  c->nranks = nranks;
  ncclResult_t r = rccl().CommInitRank(&c->comm, nranks, uid, rank);
  if (r != ncclSuccess) {
    delete c;
    return set_err(QLDPC_EHIP, std::string("ncclCommInitRank: ") + rccl().GetErrorString(r));
  }
  *out = c;
  return 0;
}

int qldpc_comm_init_all(int32_t ndev, const int32_t* devices, qldpc_comm** out) {
  if (!out || ndev < 1) return set_err(QLDPC_EINVAL, "ndev < 1 or out is NULL");
  if (int rc = need_rccl()) return rc;
  std::vector<int> devs(ndev);
  for (int i = 0; i < ndev; ++i) devs[i] = devices ? devices[i] : i;
  std::vector<ncclComm_t> comms(ndev, nullptr);
  QLDPC_RCCL(rccl().CommInitAll(comms.data(), ndev, devs.data()));
  for (int i = 0; i < ndev; ++i) {
    out[i] = new qldpc_comm();
    out[i]->comm = comms[i];
    out[i]->device = devs[i];
    out[i]->rank = i;
    out[i]->nranks = ndev;
  }
  return 0;
}

int qldpc_comm_rank(const qldpc_comm* c, int32_t* rank, int32_t* nranks, int32_t* device) {
  if (!c) return set_err(QLDPC_EINVAL, "NULL comm");
  if (rank) *rank = c->rank;
  if (nranks) *nranks = c->nranks;
  if (device) *device = c->device;
  return 0;
}

int qldpc_comm_allreduce_counters(qldpc_comm* c, void* d_counters, void* stream) {
  if (!c || !d_counters) return set_err(QLDPC_EINVAL, "NULL argument");
  QLDPC_HIP(hipSetDevice(c->device));
  QLDPC_RCCL(rccl().AllReduce(d_counters, d_counters, kCounterWords, ncclInt64, ncclSum, c->comm, (hipStream_t)stream));
  return 0;
}

int qldpc_comm_allreduce_counters_group(qldpc_comm** comms, void** d_counters, void** streams, int32_t n) {
  if (!comms || !d_counters || n < 1) return set_err(QLDPC_EINVAL, "NULL argument");
  for (int i = 0; i < n; ++i)
    if (!comms[i] || !d_counters[i]) return set_err(QLDPC_EINVAL, "NULL comm or counter buffer");
  QLDPC_RCCL(rccl().GroupStart());
  for (int i = 0; i < n; ++i) {
    (void)hipSetDevice(comms[i]->device);
    ncclResult_t r = rccl().AllReduce(d_counters[i], d_counters[i], kCounterWords, ncclInt64, ncclSum, comms[i]->comm,
                                      streams ? (hipStream_t)streams[i] : (hipStream_t) nullptr);
    if (r != ncclSuccess) {
      (void)rccl().GroupEnd();
      return set_err(QLDPC_EHIP, std::string("ncclAllReduce: ") + rccl().GetErrorString(r));
    }
  }
  QLDPC_RCCL(rccl().GroupEnd());
  return 0;
}

int qldpc_comm_destroy(qldpc_comm* c) {
  if (!c) return 0;
  if (c->comm && rccl().ok) (void)rccl().CommDestroy(c->comm);
  delete c;
  return 0;
}

int qldpc_shard_range(int64_t total, int32_t nparts, int32_t part, int64_t* begin, int64_t* count) {
  if (!begin || !count || total < 0 || nparts < 1 || part < 0 || part >= nparts)
    return set_err(QLDPC_EINVAL, "bad shard_range argument");
  // parallel.shard_range: blocks of base or base + 1 shots, the first `extra` parts one longer
  const int64_t base = total / nparts, extra = total % nparts;
  *begin = part * base + std::min<int64_t>(part, extra);
  *count = base + (part < extra ? 1 : 0);
  return 0;
}

int qldpc_mc_run_sharded(qldpc_mc** mcs, qldpc_comm** comms, int32_t ndev, double px, double py, double pz,
                         uint64_t seed, uint64_t shot_begin, int64_t shot_count, int32_t logical_mode,
                         qldpc_counters* out) {
  if (!mcs || !out || ndev < 1 || shot_count < 0) return set_err(QLDPC_EINVAL, "bad argument");
  std::vector<int> devs(ndev, 0);
  for (int d = 0; d < ndev; ++d) {
    if (!mcs[d] || !(mcs[d]->dec[0] || mcs[d]->dec[1])) return set_err(QLDPC_EINVAL, "NULL MC handle");
    devs[d] = (mcs[d]->dec[0] ? mcs[d]->dec[0] : mcs[d]->dec[1])->g->device;
    // only qldpc_comm_init_all communicators, in device order: rank d of ndev on MC handle d's
    // device (per-process init_rank communicators would sum other processes' counters into
    // shot blocks split by ndev, not by global rank)
    if (comms && (!comms[d] || comms[d]->nranks != ndev || comms[d]->rank != d))
      return set_err(QLDPC_EINVAL, "comms[d] must be rank d of an ndev-rank qldpc_comm_init_all communicator");
    if (comms && comms[d]->device != devs[d])
      return set_err(QLDPC_EINVAL, "MC handle d and communicator d are on different devices");
  }
  std::vector<void*> cnt(ndev, nullptr), streams(ndev, nullptr);
  std::vector<int> rcs(ndev, 0);
  std::vector<std::string> why(ndev);
  auto cleanup = [&] {
    for (int d = 0; d < ndev; ++d) {
      (void)hipSetDevice(devs[d]);
      if (cnt[d]) (void)hipFree(cnt[d]);
      if (streams[d]) (void)hipStreamDestroy((hipStream_t)streams[d]);
    }
  };
  // device d owns a contiguous block of global shots (parallel.shard_range).  Each device is
  // driven from its own host thread: with BP+OSD (qldpc_mc_set_osd) a launch is synchronous
  // (it reads the OSD candidate counts back), so one thread would run the devices one after
  // another.
  auto run_one = [&](int d) {
    hipError_t e = hipSetDevice(devs[d]);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(reinterpret_cast<hipStream_t*>(&streams[d]), hipStreamNonBlocking);
    if (e == hipSuccess) e = hipMalloc(&cnt[d], sizeof(qldpc_counters));
    if (e == hipSuccess) e = hipMemsetAsync(cnt[d], 0, sizeof(qldpc_counters), (hipStream_t)streams[d]);
    if (e != hipSuccess) {
      rcs[d] = QLDPC_EHIP;
      why[d] = std::string("qldpc_mc_run_sharded setup: ") + hipGetErrorString(e);
      return;
    }
    int64_t lo = 0, cnt_d = 0;
    (void)qldpc_shard_range(shot_count, ndev, d, &lo, &cnt_d);
    rcs[d] = qldpc_mc_launch(mcs[d], px, py, pz, seed, shot_begin + (uint64_t)lo, cnt_d, logical_mode, nullptr, cnt[d],
                             nullptr, nullptr, nullptr, nullptr, 0, streams[d]);
    if (rcs[d]) why[d] = qldpc_last_error();  // thread-local: carried to the caller's thread
  };
  if (ndev == 1) {
    run_one(0);
  } else {
    std::vector<std::thread> th;
    th.reserve(ndev);
    for (int d = 0; d < ndev; ++d) th.emplace_back(run_one, d);
    for (auto& t : th) t.join();
  }
  for (int d = 0; d < ndev; ++d)
    if (rcs[d]) {
      cleanup();
      return set_err(rcs[d], why[d]);
    }
  if (ndev > 1 && comms) {
    int rc = qldpc_comm_allreduce_counters_group(comms, cnt.data(), streams.data(), ndev);
    if (rc) {
      cleanup();
      return rc;
    }
  }
  // with communicators every device holds the sum (read device 0's); without, sum on the host
  const int nread = (ndev > 1 && comms) ? 1 : ndev;
  std::vector<qldpc_counters> c(nread);
  hipError_t e = hipSuccess;
  for (int d = 0; d < nread && e == hipSuccess; ++d) {
    e = hipSetDevice(devs[d]);
    if (e == hipSuccess) e = hipMemcpyAsync(&c[d], cnt[d], sizeof(qldpc_counters), hipMemcpyDeviceToHost, (hipStream_t)streams[d]);
  }
  for (int d = 0; d < ndev && e == hipSuccess; ++d) {
    e = hipSetDevice(devs[d]);
    if (e == hipSuccess) e = hipStreamSynchronize((hipStream_t)streams[d]);
  }
  cleanup();
  if (e != hipSuccess) return set_err(QLDPC_EHIP, std::string("qldpc_mc_run_sharded: ") + hipGetErrorString(e));
  int64_t* dst = reinterpret_cast<int64_t*>(out);
  for (int d = 0; d < nread; ++d) {
    const int64_t* src = reinterpret_cast<const int64_t*>(&c[d]);
    for (size_t w = 0; w < kCounterWords; ++w) dst[w] += src[w];
  }
  return 0;
}

int qldpc_sample_errors(double px, double py, double pz, uint64_t seed, uint64_t shot_begin, int64_t shot_count,
                        int32_t n, const double* d_uniforms, uint8_t* d_err, void* stream) {
  if (!d_err || n <= 0) return set_err(QLDPC_EINVAL, "NULL d_err or n <= 0");
  if (!(px >= 0 && py >= 0 && pz >= 0)) return set_err(QLDPC_EINVAL, "negative Pauli probability");
  if (shot_count <= 0) return 0;
  // thresholds in the evaluation order of src/Simulators.py:102-108 (as qldpc_mc_launch)
  const double t1 = pz, t2 = pz + px, t3 = (pz + px) + py;
  const long long total = shot_count * (long long)n;
  const int TB = 256;
  const long long grid = (total + TB - 1) / TB;
  if (grid > 0x7fffffffLL) return set_err(QLDPC_EINVAL, "too many (shot, qubit) pairs for one launch");
  hipLaunchKernelGGL(sample_errors_kernel, dim3((unsigned)grid), dim3(TB), 0, (hipStream_t)stream, seed, shot_begin,
                     (long long)shot_count, n, d_uniforms, t1, t2, t3, ceil53(t1), ceil53(t2), ceil53(t3), d_err);
  QLDPC_HIP(hipGetLastError());
  return 0;
}

int qldpc_stream_sync(void* stream) {
  QLDPC_HIP(hipStreamSynchronize((hipStream_t)stream));
  return 0;
}

}  // extern "C"
