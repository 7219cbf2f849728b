// pp3_comm.hip -- multi-GPU env shards: the one collective of the hot path.
//
// Envs are independent, so every GPU steps its own contiguous shard with no exchange inside
// the step.  The only data-path collective is the optional per-step hand-over of the
// learner batch obs | reward | done (BASELINE.json north_star: "a single RCCL gather over
// xGMI for the returned batch"):
//
//   pack_kernel   the shard's rows [nmax][D + 2] (obs, reward, done; rows past the shard's
//                 env count zero-padded so every rank contributes the same count), read from
//                 the env's device fields on the env's stream -- no host synchronisation;
//   gather        root >= 0: grouped ncclSend / ncclRecv to the learner rank (each peer's
//                 chunk crosses its own xGMI link to the root once -- a point-to-point mesh,
//                 so no ring relay); root < 0: ncclAllGather (every rank gets the batch).
//
// RCCL is loaded lazily with dlopen (librccl.so.1 from /opt/rocm/lib), so the single-GPU path
// never maps it.  The unique id is created by rank 0 (pp3_comm_unique_id) and handed to the
// other ranks out of band (pupperv3_mjx/sharding.py: a file rendezvous on the node).  No torch.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <string.h>

#include <mutex>
#include <string>

#include "pupper_hip.h"

namespace {

struct Rccl {
  void* so = nullptr;
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*AllGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*AllReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  const char* (*GetErrorString)(ncclResult_t) = nullptr;
};

thread_local std::string g_cerr;
int cerr(int code, const std::string& m) {
  g_cerr = m;
  return code;
}

// loaded once per process (std::call_once: safe from several host threads); a failure is
// remembered and reported to every caller
Rccl g_rccl;
std::string g_rccl_err;
void load_rccl() {
  Rccl& r = g_rccl;
#ifdef PP3_TEST_RCCL_SONAME
  // test build only (`make loopback` -> tests/loopback/, never the product library): the RCCL API
  // of the loopback test transport built next to this library (several rank processes on one
  // GPU, which RCCL refuses); pp3_create refuses this build unless the caller opts in (pp3_diag.h)
  Dl_info self;
  std::string path = PP3_TEST_RCCL_SONAME;
  if (dladdr((const void*)&load_rccl, &self) && self.dli_fname) {
    const std::string me = self.dli_fname;
    const size_t cut = me.rfind('/');
    if (cut != std::string::npos) path = me.substr(0, cut + 1) + PP3_TEST_RCCL_SONAME;
  }
  const char* names[] = {path.c_str()};
#else
  const char* names[] = {"librccl.so.1", "/opt/rocm/lib/librccl.so.1", "librccl.so"};
#endif
  for (const char* n : names)
    if ((r.so = dlopen(n, RTLD_NOW | RTLD_LOCAL)) != nullptr) break;
  if (!r.so) {
    g_rccl_err = std::string("cannot load librccl.so.1: ") + dlerror();
    return;
  }
#define SYM(field, name)                                                          \
  r.field = reinterpret_cast<decltype(r.field)>(dlsym(r.so, name));               \
  if (!r.field) {                                                                 \
    g_rccl_err = std::string("librccl.so.1 lacks ") + name;                       \
    r.so = nullptr;                                                               \
    return;                                                                       \
  }
  SYM(GetUniqueId, "ncclGetUniqueId")
  SYM(CommInitRank, "ncclCommInitRank")
  SYM(CommDestroy, "ncclCommDestroy")
  SYM(AllGather, "ncclAllGather")
  SYM(AllReduce, "ncclAllReduce")
  SYM(Send, "ncclSend")
  SYM(Recv, "ncclRecv")
  SYM(GroupStart, "ncclGroupStart")
  SYM(GroupEnd, "ncclGroupEnd")
  SYM(GetErrorString, "ncclGetErrorString")
#undef SYM
}
const Rccl* rccl() {
  static std::once_flag once;
  std::call_once(once, load_rccl);
  if (!g_rccl.so) {
    g_cerr = g_rccl_err;
    return nullptr;
  }
  return &g_rccl;
}

// sets `device` current for the scope and restores the caller's device on exit
struct DeviceScope {
  int prev = -1;
  hipError_t err;
  explicit DeviceScope(int device) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    err = hipSetDevice(device);
  }
  ~DeviceScope() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

#define HCHK(x)                                                                                   \
  do {                                                                                            \
    hipError_t e_ = (x);                                                                          \
    if (e_ != hipSuccess) return cerr(PP3_ERR_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)
#define NCHK(R, x)                                                                                  \
  do {                                                                                              \
    ncclResult_t r_ = (x);                                                                          \
    if (r_ != ncclSuccess) return cerr(PP3_ERR_COMM, std::string(#x) + ": " + (R)->GetErrorString(r_)); \
  } while (0)

// learner rows of one shard: out[row][0:D] = obs, [D] = reward, [D+1] = done; rows >= n zero.
// One thread per output float (coalesced in both the obs reads and the packed writes).
__global__ void pack_kernel(const float* __restrict__ obs, const float* __restrict__ rew,
                            const float* __restrict__ done, int n, int D, int nmax, float* __restrict__ out) {
  const int W = D + 2;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)nmax * W) return;
  const int row = (int)(i / W), c = (int)(i - (long)row * W);
  float v = 0.0f;
  if (row < n) v = c < D ? obs[(long)row * D + c] : (c == D ? rew[row] : done[row]);
  out[i] = v;
}

// the same for a K-step trajectory ([K][n][D] obs, [K][n] reward / done) -> out [K][nmax][D + 2]
__global__ void pack_traj_kernel(const float* __restrict__ obs, const float* __restrict__ rew,
                                 const float* __restrict__ done, int n, int D, int nmax, long total,
                                 float* __restrict__ out) {
  const int W = D + 2;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const long per = (long)nmax * W;
  const long t = i / per;
  const long j = i - t * per;
  const int row = (int)(j / W), c = (int)(j - (long)row * W);
  float v = 0.0f;
  if (row < n) {
    const long r = t * n + row;
    v = c < D ? obs[r * D + c] : (c == D ? rew[r] : done[r]);
  }
  out[i] = v;
}

}  // namespace

struct pp3_comm {
  int rank, world, device;
  ncclComm_t comm;
  hipStream_t stream;  // host-blocking helpers (barrier, reductions)
  float* pack;         // [nmax][D+2] (or [K][nmax][D+2]) staging of this rank's chunk (allgather / non-root)
  size_t pack_elems;
  double* red;         // reduction scratch
};
namespace {
int exchange(pp3_comm* c, const Rccl* R, float* mine, size_t count, int root, float* dst_dev, hipStream_t s);
// where this rank's chunk of `count` floats is packed: the root straight into its own slot of the
// destination, every other rank into the (grown on demand) staging buffer
int chunk_of(pp3_comm* c, size_t count, int root, float* dst_dev, hipStream_t s, float** mine) {
  if (root >= 0 && root == c->rank) {
    *mine = dst_dev + (size_t)c->rank * count;
    return PP3_OK;
  }
  if (c->pack_elems < count) {
    HCHK(hipStreamSynchronize(s));  // (first call / growth only) the old buffer may be in flight
    (void)hipFree(c->pack);
    c->pack = nullptr;
    HCHK(hipMalloc(&c->pack, count * sizeof(float)));
    c->pack_elems = count;
  }
  *mine = c->pack;
  return PP3_OK;
}
}  // namespace

extern "C" {

const char* pp3_comm_last_error(void) { return g_cerr.c_str(); }

int pp3_comm_unique_id(uint8_t* out) {
  if (!out) return cerr(PP3_ERR_ARG, "pp3_comm_unique_id: null output");
  const Rccl* R = rccl();
  if (!R) return cerr(PP3_ERR_COMM, g_cerr);
  ncclUniqueId id;
  NCHK(R, R->GetUniqueId(&id));
  static_assert(sizeof(id) == PP3_COMM_ID_BYTES, "ncclUniqueId size");
  memcpy(out, &id, sizeof(id));
  return PP3_OK;
}

int pp3_comm_init(const uint8_t* id, int32_t rank, int32_t world, int32_t device, pp3_comm_t** out) {
  if (!id || !out || world < 1 || rank < 0 || rank >= world) return cerr(PP3_ERR_ARG, "pp3_comm_init: bad argument");
  const Rccl* R = rccl();
  if (!R) return cerr(PP3_ERR_COMM, g_cerr);
  DeviceScope dev(device);
  HCHK(dev.err);
  ncclUniqueId uid;
  memcpy(&uid, id, sizeof(uid));
  pp3_comm* c = new pp3_comm();
  memset(c, 0, sizeof(*c));
  c->rank = rank;
  c->world = world;
  c->device = device;
  ncclResult_t r = R->CommInitRank(&c->comm, world, uid, rank);
  if (r != ncclSuccess) {
    delete c;
    return cerr(PP3_ERR_COMM, std::string("ncclCommInitRank: ") + R->GetErrorString(r));
  }
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipMalloc(&c->red, 64 * sizeof(double)) != hipSuccess) {
    R->CommDestroy(c->comm);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return cerr(PP3_ERR_HIP, "pp3_comm_init: stream / scratch allocation failed");
  }
  *out = c;
  return PP3_OK;
}

int pp3_comm_destroy(pp3_comm_t* c) {
  if (!c) return PP3_OK;
  const Rccl* R = rccl();
  DeviceScope dev(c->device);
  (void)hipStreamSynchronize(c->stream);
  if (R) R->CommDestroy(c->comm);
  (void)hipFree(c->pack);
  (void)hipFree(c->red);
  (void)hipStreamDestroy(c->stream);
  delete c;
  return PP3_OK;
}

int32_t pp3_comm_rank(const pp3_comm_t* c) { return c ? c->rank : -1; }
int32_t pp3_comm_world(const pp3_comm_t* c) { return c ? c->world : 0; }

int pp3_gather(pp3_comm_t* c, pp3_env_t* e, int32_t nmax, int32_t root, float* dst_dev, void* stream) {
  if (!c || !e) return cerr(PP3_ERR_ARG, "pp3_gather: null argument");
  if (root >= c->world) return cerr(PP3_ERR_ARG, "pp3_gather: root out of range");
  if (pp3_env_device(e) != c->device)
    return cerr(PP3_ERR_ARG, "pp3_gather: the env and the communicator are on different devices");
  const int n = pp3_num_envs(e);
  if (nmax < n) return cerr(PP3_ERR_ARG, "pp3_gather: nmax smaller than this rank's shard");
  if ((root < 0 || root == c->rank) && !dst_dev) return cerr(PP3_ERR_ARG, "pp3_gather: null destination");
  const Rccl* R = rccl();
  if (!R) return cerr(PP3_ERR_COMM, g_cerr);
  void *obs, *rew, *done;
  int64_t D, one;
  if (pp3_field(e, PP3_F_OBS, &obs, &D) || pp3_field(e, PP3_F_REWARD, &rew, &one) ||
      pp3_field(e, PP3_F_DONE, &done, &one))
    return cerr(PP3_ERR_ARG, std::string("pp3_gather: ") + pp3_last_error());
  const size_t W = (size_t)D + 2, count = (size_t)nmax * W;
  hipStream_t s = stream ? (hipStream_t)stream : (hipStream_t)pp3_stream(e);
  DeviceScope dev(c->device);
  HCHK(dev.err);
  float* mine;
  if (const int rc = chunk_of(c, count, root, dst_dev, s, &mine)) return rc;
  const unsigned blocks = (unsigned)((count + 255) / 256);
  hipLaunchKernelGGL(pack_kernel, dim3(blocks), dim3(256), 0, s, (const float*)obs, (const float*)rew,
                     (const float*)done, n, (int)D, nmax, mine);
  HCHK(hipGetLastError());
  return exchange(c, R, mine, count, root, dst_dev, s);
}

int pp3_gather_rollout(pp3_comm_t* c, pp3_env_t* e, const float* traj_obs, const float* traj_reward,
                       const float* traj_done, int32_t nsteps, int32_t nmax, int32_t root, float* dst_dev,
                       void* stream) {
  if (!c || !e || !traj_obs || !traj_reward || !traj_done) return cerr(PP3_ERR_ARG, "pp3_gather_rollout: null argument");
  if (nsteps < 1) return cerr(PP3_ERR_ARG, "pp3_gather_rollout: nsteps must be >= 1");
  if (root >= c->world) return cerr(PP3_ERR_ARG, "pp3_gather_rollout: root out of range");
  if (pp3_env_device(e) != c->device)
    return cerr(PP3_ERR_ARG, "pp3_gather_rollout: the env and the communicator are on different devices");
  const int n = pp3_num_envs(e);
  if (nmax < n) return cerr(PP3_ERR_ARG, "pp3_gather_rollout: nmax smaller than this rank's shard");
  if ((root < 0 || root == c->rank) && !dst_dev) return cerr(PP3_ERR_ARG, "pp3_gather_rollout: null destination");
  const Rccl* R = rccl();
  if (!R) return cerr(PP3_ERR_COMM, g_cerr);
  void* obs;
  int64_t D;
  if (pp3_field(e, PP3_F_OBS, &obs, &D)) return cerr(PP3_ERR_ARG, std::string("pp3_gather_rollout: ") + pp3_last_error());
  const size_t W = (size_t)D + 2, count = (size_t)nsteps * nmax * W;
  hipStream_t s = stream ? (hipStream_t)stream : (hipStream_t)pp3_stream(e);
  DeviceScope dev(c->device);
  HCHK(dev.err);
  float* mine;
  if (const int rc = chunk_of(c, count, root, dst_dev, s, &mine)) return rc;
  const unsigned blocks = (unsigned)((count + 255) / 256);
  hipLaunchKernelGGL(pack_traj_kernel, dim3(blocks), dim3(256), 0, s, traj_obs, traj_reward, traj_done, n, (int)D,
                     nmax, (long)count, mine);
  HCHK(hipGetLastError());
  return exchange(c, R, mine, count, root, dst_dev, s);
}

}  // extern "C"

namespace {
// the collective of pp3_gather / pp3_gather_rollout: this rank's `count` floats at `mine` (already
// in its own slot when it is the root) -> rank-major slots of `count` at dst
int exchange(pp3_comm* c, const Rccl* R, float* mine, size_t count, int root, float* dst_dev, hipStream_t s) {
  if (root < 0) {
    NCHK(R, R->AllGather(mine, dst_dev, count, ncclFloat32, c->comm, s));
  } else if (c->world > 1) {
    NCHK(R, R->GroupStart());
    if (c->rank == root) {
      for (int r = 0; r < c->world; r++)
        if (r != root) {
          ncclResult_t rr = R->Recv(dst_dev + (size_t)r * count, count, ncclFloat32, r, c->comm, s);
          if (rr != ncclSuccess) { R->GroupEnd(); return cerr(PP3_ERR_COMM, std::string("ncclRecv: ") + R->GetErrorString(rr)); }
        }
    } else {
      ncclResult_t rr = R->Send(mine, count, ncclFloat32, root, c->comm, s);
      if (rr != ncclSuccess) { R->GroupEnd(); return cerr(PP3_ERR_COMM, std::string("ncclSend: ") + R->GetErrorString(rr)); }
    }
    NCHK(R, R->GroupEnd());
  }
  return PP3_OK;
}
}  // namespace

extern "C" {

int pp3_comm_allreduce(pp3_comm_t* c, const double* in, double* out, int32_t n, int32_t op) {
  if (!c || !in || !out || n < 1 || n > 64) return cerr(PP3_ERR_ARG, "pp3_comm_allreduce: bad argument (n <= 64)");
  const Rccl* R = rccl();
  if (!R) return cerr(PP3_ERR_COMM, g_cerr);
  DeviceScope dev(c->device);
  HCHK(dev.err);
  HCHK(hipMemcpyAsync(c->red, in, n * sizeof(double), hipMemcpyHostToDevice, c->stream));
  NCHK(R, R->AllReduce(c->red, c->red, n, ncclFloat64, op == PP3_REDUCE_MAX ? ncclMax : ncclSum, c->comm, c->stream));
  HCHK(hipMemcpyAsync(out, c->red, n * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  HCHK(hipStreamSynchronize(c->stream));
  return PP3_OK;
}

int pp3_comm_barrier(pp3_comm_t* c) {
  double z = 0.0, o = 0.0;
  return pp3_comm_allreduce(c, &z, &o, 1, PP3_REDUCE_SUM);
}

}  // extern "C"
