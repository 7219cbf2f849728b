// loopback_rccl.cpp -- TEST TRANSPORT ONLY: the subset of the RCCL API that pp3_comm.hip calls,
// implemented between processes that all share ONE GPU, so the multi-rank code paths (several
// rank processes, pp3_gather's grouped send/recv to a root and its all-gather, the all-reduce
// behind the bench's barrier and max-over-ranks timing, bench.py's gather_check) run on the
// one-GPU test pool.  Real RCCL refuses two ranks on one device.
//
// Loaded only when PP3_RCCL_LIBRARY names it (pp3_comm.hip load_rccl); the product path always
// loads librccl.  Every operation is blocking and host-staged: it synchronises the caller's
// stream, moves the payload through files in a per-communicator directory, and copies the
// received bytes to the device before returning -- the semantics RCCL guarantees once the
// stream has drained, without its asynchrony.  It exercises the callers' argument and placement
// logic, not RCCL's transport.
//
// Layout of a communicator's directory (name carried in the ncclUniqueId, made by rank 0):
//   p2p.<src>.<dst>.<k>   the k-th send from src to dst (the receiver deletes it)
//   coll.<k>.<rank>       rank's contribution to the k-th collective (deleted two rounds later:
//                         by then every rank has read it)
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <chrono>
#include <string>
#include <thread>
#include <vector>

struct ncclComm {
  std::string dir;
  int rank, world;
  long coll;                      // collectives issued so far (same order on every rank)
  std::vector<long> sent, recvd;  // point-to-point messages per peer
};

namespace {

constexpr double kTimeoutS = 120.0;

size_t type_size(ncclDataType_t t) {
  switch (t) {
    case ncclInt8: case ncclUint8: return 1;
    case ncclFloat16: case ncclBfloat16: return 2;
    case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
    case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
    default: return 0;
  }
}

bool write_file(const std::string& path, const void* data, size_t bytes) {
  const std::string tmp = path + ".tmp";
  FILE* f = fopen(tmp.c_str(), "wb");
  if (!f) return false;
  const bool ok = fwrite(data, 1, bytes, f) == bytes;
  if (fclose(f) != 0 || !ok) return false;
  return rename(tmp.c_str(), path.c_str()) == 0;  // atomic publish
}

// polls until `path` exists, then reads exactly `bytes`
bool read_file(const std::string& path, void* data, size_t bytes) {
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    FILE* f = fopen(path.c_str(), "rb");
    if (f) {
      const size_t got = fread(data, 1, bytes, f);
      fclose(f);
      return got == bytes;
    }
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > kTimeoutS) return false;
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

std::string coll_path(const ncclComm* c, long k, int r) {
  return c->dir + "/coll." + std::to_string(k) + "." + std::to_string(r);
}

// one all-to-all exchange of equal-size host blocks: out[r] = rank r's block
ncclResult_t exchange(ncclComm* c, const void* mine, size_t bytes, std::vector<char>& out) {
  const long k = c->coll++;
  if (!write_file(coll_path(c, k, c->rank), mine, bytes)) return ncclSystemError;
  out.resize(bytes * c->world);
  for (int r = 0; r < c->world; r++)
    if (!read_file(coll_path(c, k, r), out.data() + bytes * r, bytes)) return ncclSystemError;
  if (k >= 2) remove(coll_path(c, k - 2, c->rank).c_str());
  return ncclSuccess;
}

}  // namespace

extern "C" {

const char* ncclGetErrorString(ncclResult_t r) {
  switch (r) {
    case ncclSuccess: return "no error";
    case ncclInvalidArgument: return "loopback: invalid argument";
    case ncclSystemError: return "loopback: file exchange failed or timed out";
    default: return "loopback: error";
  }
}

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
  if (!id) return ncclInvalidArgument;
  memset(id, 0, sizeof(*id));
  const char* base = getenv("PP3_LOOPBACK_DIR");
  snprintf(id->internal, sizeof(id->internal), "%s/pp3_loopback_%d_%lld", base ? base : "/tmp", (int)getpid(),
           (long long)std::chrono::steady_clock::now().time_since_epoch().count());
  return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId id, int rank) {
  if (!comm || nranks < 1 || rank < 0 || rank >= nranks || !id.internal[0]) return ncclInvalidArgument;
  std::string dir(id.internal, strnlen(id.internal, sizeof(id.internal)));
  if (mkdir(dir.c_str(), 0700) != 0 && errno != EEXIST) return ncclSystemError;
  ncclComm* c = new ncclComm();
  c->dir = dir;
  c->rank = rank;
  c->world = nranks;
  c->coll = 0;
  c->sent.assign(nranks, 0);
  c->recvd.assign(nranks, 0);
  std::vector<char> all;  // every rank has joined before the init returns (as in RCCL)
  const char one = 1;
  if (exchange(c, &one, 1, all) != ncclSuccess) {
    delete c;
    return ncclSystemError;
  }
  *comm = c;
  return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t c) {
  if (!c) return ncclSuccess;
  for (long k = c->coll - 2; k < c->coll; k++)
    if (k >= 0) remove(coll_path(c, k, c->rank).c_str());
  rmdir(c->dir.c_str());  // (succeeds for the last rank to leave)
  delete c;
  return ncclSuccess;
}

ncclResult_t ncclGroupStart() { return ncclSuccess; }
ncclResult_t ncclGroupEnd() { return ncclSuccess; }

// sends never wait for their receiver, so a grouped pattern of sends and receives cannot deadlock
ncclResult_t ncclSend(const void* buf, size_t count, ncclDataType_t dt, int peer, ncclComm_t c, hipStream_t s) {
  const size_t bytes = count * type_size(dt);
  if (!c || !buf || !bytes || peer < 0 || peer >= c->world || peer == c->rank) return ncclInvalidArgument;
  std::vector<char> h(bytes);
  if (hipStreamSynchronize(s) != hipSuccess || hipMemcpy(h.data(), buf, bytes, hipMemcpyDeviceToHost) != hipSuccess)
    return ncclSystemError;
  const std::string p = c->dir + "/p2p." + std::to_string(c->rank) + "." + std::to_string(peer) + "." +
                        std::to_string(c->sent[peer]++);
  return write_file(p, h.data(), bytes) ? ncclSuccess : ncclSystemError;
}

ncclResult_t ncclRecv(void* buf, size_t count, ncclDataType_t dt, int peer, ncclComm_t c, hipStream_t s) {
  const size_t bytes = count * type_size(dt);
  if (!c || !buf || !bytes || peer < 0 || peer >= c->world || peer == c->rank) return ncclInvalidArgument;
  const std::string p = c->dir + "/p2p." + std::to_string(peer) + "." + std::to_string(c->rank) + "." +
                        std::to_string(c->recvd[peer]++);
  std::vector<char> h(bytes);
  if (!read_file(p, h.data(), bytes)) return ncclSystemError;
  remove(p.c_str());
  if (hipStreamSynchronize(s) != hipSuccess || hipMemcpy(buf, h.data(), bytes, hipMemcpyHostToDevice) != hipSuccess)
    return ncclSystemError;
  return ncclSuccess;
}

ncclResult_t ncclAllGather(const void* send, void* recv, size_t count, ncclDataType_t dt, ncclComm_t c, hipStream_t s) {
  const size_t bytes = count * type_size(dt);
  if (!c || !send || !recv || !bytes) return ncclInvalidArgument;
  std::vector<char> h(bytes), all;
  if (hipStreamSynchronize(s) != hipSuccess || hipMemcpy(h.data(), send, bytes, hipMemcpyDeviceToHost) != hipSuccess)
    return ncclSystemError;
  const ncclResult_t r = exchange(c, h.data(), bytes, all);
  if (r != ncclSuccess) return r;
  return hipMemcpy(recv, all.data(), all.size(), hipMemcpyHostToDevice) == hipSuccess ? ncclSuccess : ncclSystemError;
}

ncclResult_t ncclAllReduce(const void* send, void* recv, size_t count, ncclDataType_t dt, ncclRedOp_t op, ncclComm_t c,
                           hipStream_t s) {
  if (!c || !send || !recv || !count || (dt != ncclFloat64 && dt != ncclFloat32) || (op != ncclSum && op != ncclMax))
    return ncclInvalidArgument;
  const size_t bytes = count * type_size(dt);
  std::vector<char> h(bytes), all;
  if (hipStreamSynchronize(s) != hipSuccess || hipMemcpy(h.data(), send, bytes, hipMemcpyDeviceToHost) != hipSuccess)
    return ncclSystemError;
  const ncclResult_t r = exchange(c, h.data(), bytes, all);
  if (r != ncclSuccess) return r;
  for (size_t i = 0; i < count; i++) {  // rank order, as a deterministic reduction
    double acc = 0.0;
    for (int q = 0; q < c->world; q++) {
      const char* p = all.data() + bytes * q;
      const double v = dt == ncclFloat64 ? ((const double*)p)[i] : (double)((const float*)p)[i];
      acc = q == 0 ? v : (op == ncclSum ? acc + v : (v > acc ? v : acc));
    }
    if (dt == ncclFloat64) ((double*)h.data())[i] = acc;
    else ((float*)h.data())[i] = (float)acc;
  }
  return hipMemcpy(recv, h.data(), bytes, hipMemcpyHostToDevice) == hipSuccess ? ncclSuccess : ncclSystemError;
}

}  // extern "C"
