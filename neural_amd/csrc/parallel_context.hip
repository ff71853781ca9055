// parallel_context.hip -- the tensor-parallel communicator of Neural Speed re-hosted on MI355X.
//
// Replaces neural_speed/core/parallel_context.{h,cpp} (oneCCL over MPI + a same-host SHM all-reduce,
// shared_memory_ccl.hpp:100-139) with the same extern "C" surface (parallel_context.h:40-48):
//   init_parallel_context / get_tp_size / get_tp_rank / is_master / barrier / broadcast / alltoall / reduce_add
// called by ne_layers.c:1672-1739 (weight split), 5466-5476 (ne_all_reduce) and 9005-9076.
//
// Transport, one process per GPU:
//   * bootstrap: a TCP rendezvous (rank 0 listens on NAD_TP_ADDR or MASTER_ADDR:MASTER_PORT+17) that all-gathers small
//     blobs -- the RCCL unique id, IPC handles, barrier tokens.  Ranks come from NAD_TP_RANK/SIZE, RANK/WORLD_SIZE
//     (torch.distributed.run), OMPI_COMM_WORLD_* or PMI_* (mpirun, like the reference), else a world of 1.
//   * large device messages: RCCL (ncclAllReduce / ncclBroadcast / ncclAllToAll) on the caller's stream (xGMI).
//   * small device all-reduces (<= NAD_PC_ONESHOT_BYTES, default 512 KiB): a one-shot kernel over IPC-mapped peer
//     buffers -- every rank publishes its slice into its own fine-grained buffer, raises a flag in every peer, waits for
//     the peers' flags and sums all ranks' slices in rank order (identical bits on every rank).  Two buffers by
//     generation parity; the generation lives on the device so the launch is graph-capturable.  Every spin is bounded
//     and reports through a device status word (nad_pc_status).
//   * host pointers (the reference's CPU tensors): staged through the device path; without a GPU (NAD_PC_TRANSPORT=tcp
//     or no HIP device) the bootstrap sockets carry them (sum in rank order at rank 0, then broadcast).
#include <arpa/inet.h>
#include <hip/hip_runtime.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <rccl/rccl.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/neural_amd.h"

namespace {

int env_int(const char* a, const char* b, const char* c, const char* d, int def) {
  for (const char* n : {a, b, c, d}) {
    if (!n) continue;
    const char* v = getenv(n);
    if (v && *v) return atoi(v);
  }
  return def;
}

void pc_log(const char* fmt, const char* what) { fprintf(stderr, "neural_amd parallel_context: %s%s\n", fmt, what); }

// ------------------------------------------------------------------------------------------------ TCP rendezvous
bool send_all(int fd, const void* p, size_t n) {
  const char* c = static_cast<const char*>(p);
  while (n) {
    ssize_t k = ::send(fd, c, n, MSG_NOSIGNAL);
    if (k <= 0) return false;
    c += k;
    n -= size_t(k);
  }
  return true;
}
bool recv_all(int fd, void* p, size_t n) {
  char* c = static_cast<char*>(p);
  while (n) {
    ssize_t k = ::recv(fd, c, n, 0);
    if (k <= 0) return false;
    c += k;
    n -= size_t(k);
  }
  return true;
}

struct Rendezvous {
  int rank = 0, world = 1;
  int listen_fd = -1;
  std::vector<int> peers;  // rank 0: fd of rank r (index r); others: peers[0] = fd to rank 0
  std::string err;

  bool open(const std::string& host, int port, int timeout_s) {
    if (world == 1) return true;
    peers.assign(size_t(world), -1);
    if (rank == 0) {
      listen_fd = ::socket(AF_INET, SOCK_STREAM, 0);
      int one = 1;
      setsockopt(listen_fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
      sockaddr_in a{};
      a.sin_family = AF_INET;
      a.sin_port = htons(uint16_t(port));
      a.sin_addr.s_addr = htonl(INADDR_ANY);
      if (::bind(listen_fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0 || ::listen(listen_fd, world) != 0) {
        err = "cannot listen on port " + std::to_string(port);
        return false;
      }
      for (int i = 1; i < world; i++) {
        int fd = ::accept(listen_fd, nullptr, nullptr);
        if (fd < 0) {
          err = "accept failed";
          return false;
        }
        setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
        int32_t r = -1;
        if (!recv_all(fd, &r, 4) || r <= 0 || r >= world || peers[size_t(r)] >= 0) {
          err = "bad rank in rendezvous hello";
          return false;
        }
        peers[size_t(r)] = fd;
      }
      return true;
    }
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    if (getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res) != 0 || !res) {
      err = "cannot resolve " + host;
      return false;
    }
    const auto t0 = std::chrono::steady_clock::now();
    int fd = -1;
    while (true) {
      fd = ::socket(AF_INET, SOCK_STREAM, 0);
      if (::connect(fd, res->ai_addr, res->ai_addrlen) == 0) break;
      ::close(fd);
      fd = -1;
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(timeout_s)) break;
      std::this_thread::sleep_for(std::chrono::milliseconds(50));
    }
    freeaddrinfo(res);
    if (fd < 0) {
      err = "cannot connect to rank 0 at " + host + ":" + std::to_string(port);
      return false;
    }
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    int32_t r = rank;
    if (!send_all(fd, &r, 4)) {
      err = "hello failed";
      return false;
    }
    peers[0] = fd;
    return true;
  }

  // every rank contributes `n` bytes; out receives world * n bytes in rank order
  bool allgather(const void* in, void* out, size_t n) {
    char* o = static_cast<char*>(out);
    std::memcpy(o + size_t(rank) * n, in, n);
    if (world == 1) return true;
    if (rank == 0) {
      for (int r = 1; r < world; r++)
        if (!recv_all(peers[size_t(r)], o + size_t(r) * n, n)) return fail("allgather recv");
      for (int r = 1; r < world; r++)
        if (!send_all(peers[size_t(r)], o, size_t(world) * n)) return fail("allgather send");
      return true;
    }
    if (!send_all(peers[0], in, n) || !recv_all(peers[0], o, size_t(world) * n)) return fail("allgather");
    return true;
  }
  bool fail(const char* what) {
    err = what;
    return false;
  }
  void close_all() {
    for (int fd : peers)
      if (fd >= 0) ::close(fd);
    peers.clear();
    if (listen_fd >= 0) ::close(listen_fd);
    listen_fd = -1;
  }
};

// ------------------------------------------------------------------------------------------------ one-shot kernel
constexpr int kMaxRanks = 16;
constexpr int kOneShotBlocks = 64;  // workgroups of the one-shot all-reduce (each owns a slice; per-slice flags)
constexpr int kOneShotThreads = 512;

struct PeerPtrs {
  float* data[kMaxRanks];     // peer r's data area: [2 parities][cap floats]
  uint32_t* flags[kMaxRanks];  // peer r's flag area: [kOneShotBlocks][kMaxRanks]
};

// gen = ctl[0] + 1 for the whole launch; the last workgroup to finish stores it back (stream order makes the next
// launch see it).  ctl[1] = finished-workgroup counter, ctl[2] = status (1 = a peer never arrived).
__global__ __launch_bounds__(kOneShotThreads) void nad_oneshot_allreduce_kernel(const float* in,
                                                                                  float* out, size_t count,
                                                                                  size_t cap, int rank, int world,
                                                                                  PeerPtrs peers, uint32_t* ctl) {
  __shared__ uint32_t s_gen;
  __shared__ int s_ok;
  if (threadIdx.x == 0) {
    s_gen = __hip_atomic_load(&ctl[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    s_ok = 1;
  }
  __syncthreads();
  const uint32_t gen = s_gen;
  const size_t par = size_t(gen & 1u) * cap;
  // this workgroup's slice, in float4 units where possible
  const size_t per = (count + gridDim.x - 1) / gridDim.x;
  const size_t lo = std::min(count, size_t(blockIdx.x) * per), hi = std::min(count, lo + per);
  float* mine = peers.data[rank] + par;
  for (size_t i = lo + threadIdx.x; i < hi; i += blockDim.x) __builtin_nontemporal_store(in[i], &mine[i]);
  __atomic_thread_fence(__ATOMIC_RELEASE);  // every wave: its slice stores are complete (system scope)
  __syncthreads();
  if (threadIdx.x < unsigned(world)) {
    // publish: my slice is in my buffer -> raise flag [block][rank] in peer threadIdx.x (system-scope release)
    uint32_t* f = peers.flags[threadIdx.x] + blockIdx.x * kMaxRanks + rank;
    __hip_atomic_store(f, gen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    // wait for peer threadIdx.x's flag in my own flag area
    const uint32_t* g = peers.flags[rank] + blockIdx.x * kMaxRanks + threadIdx.x;
    long spins = 0;
    while (__hip_atomic_load(g, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != gen) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > (1l << 26)) {
        s_ok = 0;
        break;
      }
    }
  }
  __syncthreads();
  __atomic_thread_fence(__ATOMIC_ACQUIRE);
  if (!s_ok) {
    if (threadIdx.x == 0) __hip_atomic_store(&ctl[2], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    for (size_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
      float s = 0.f;
      for (int r = 0; r < world; r++) s += __builtin_nontemporal_load(&peers.data[r][par + i]);  // rank order
      out[i] = s;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t done = __hip_atomic_fetch_add(&ctl[1], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    if (done == gridDim.x) {
      __hip_atomic_store(&ctl[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&ctl[0], gen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

}  // namespace

// ------------------------------------------------------------------------------------------------ the context
struct parallel_context {
  int rank = 0, world = 1, local_rank = 0, device = -1;
  bool gpu = false;       // HIP device present and used
  bool use_rccl = true;   // NAD_PC_NO_RCCL=1: one-shot + staging only (e.g. several ranks on one GPU in tests)
  bool force_rccl = false;  // NAD_PC_FORCE_RCCL=1: RCCL communicator and RCCL all-reduce even at world 1 (tests)
  Rendezvous rv;
  ncclComm_t comm = nullptr;
  hipStream_t stream = nullptr;  // stream of the reference entry points (nad_pc_set_stream); NULL = the null stream
  // one-shot all-reduce
  size_t oneshot_cap = 0;        // floats per parity
  void* own = nullptr;           // [2][cap] floats + flags
  std::vector<void*> opened;     // IPC-mapped peer buffers
  PeerPtrs peers{};
  uint32_t* ctl = nullptr;
  bool oneshot = false;
  bool oneshot_uncached = false;  // the one-shot buffer is fine-grained uncached memory (else the hipMalloc fallback)
  // host staging
  float* stage = nullptr;
  size_t stage_bytes = 0;
  std::mutex mu;
  std::string err;
};

namespace {
parallel_context* g_ctx = nullptr;
std::mutex g_ctx_mu;

void set_pc_err(parallel_context* p, const std::string& e) {
  p->err = e;
  pc_log("", e.c_str());
}

bool rccl_init(parallel_context* p) {
  if (p->comm || !p->use_rccl || (p->world == 1 && !p->force_rccl)) return p->comm != nullptr || p->world == 1;
  ncclUniqueId id{};
  if (p->rank == 0 && ncclGetUniqueId(&id) != ncclSuccess) {
    set_pc_err(p, "ncclGetUniqueId failed");
    return false;
  }
  std::vector<ncclUniqueId> all(size_t(p->world));
  if (!p->rv.allgather(&id, all.data(), sizeof(id))) {
    set_pc_err(p, "rendezvous: " + p->rv.err);
    return false;
  }
  if (ncclCommInitRank(&p->comm, p->world, all[0], p->rank) != ncclSuccess) {
    set_pc_err(p, "ncclCommInitRank failed");
    p->comm = nullptr;
    return false;
  }
  return true;
}

bool oneshot_init(parallel_context* p) {
  if (p->world == 1 || !p->gpu || p->world > kMaxRanks) return false;
  const int bytes = env_int("NAD_PC_ONESHOT_BYTES", nullptr, nullptr, nullptr, 512 * 1024);
  if (bytes <= 0) return false;
  p->oneshot_cap = (size_t(bytes) / 4 + 63) / 64 * 64;
  const size_t flag_bytes = size_t(kOneShotBlocks) * kMaxRanks * 4;
  const size_t total = 2 * p->oneshot_cap * 4 + flag_bytes;
  // fine-grained uncached memory (flags and slices bypass the caches); plain device memory if that cannot be shared
  hipIpcMemHandle_t h{};
  bool have = false;
  for (int attempt = 0; attempt < 2 && !have; attempt++) {
    hipError_t e = attempt == 0 ? hipExtMallocWithFlags(&p->own, total, hipDeviceMallocUncached)
                                : hipMalloc(&p->own, total);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      p->own = nullptr;
      continue;
    }
    if (hipIpcGetMemHandle(&h, p->own) == hipSuccess) {
      have = true;
      p->oneshot_uncached = attempt == 0;
    } else {
      (void)hipGetLastError();
      (void)hipFree(p->own);
      p->own = nullptr;
    }
  }
  int okh = have ? 1 : 0;
  std::vector<int> okhs(size_t(p->world));
  if (!p->rv.allgather(&okh, okhs.data(), sizeof(int))) return false;
  for (int v : okhs) okh &= v;
  if (!okh) {
    set_pc_err(p, "hipIpcGetMemHandle failed on some rank: one-shot all-reduce disabled");
    return false;
  }
  if (hipMemset(p->own, 0, total) != hipSuccess || hipMalloc(&p->ctl, 64) != hipSuccess ||
      hipMemset(p->ctl, 0, 64) != hipSuccess || hipDeviceSynchronize() != hipSuccess)
    return false;
  std::vector<hipIpcMemHandle_t> all(size_t(p->world));
  if (!p->rv.allgather(&h, all.data(), sizeof(h))) return false;
  int ok = 1;
  for (int r = 0; r < p->world; r++) {
    void* base = p->own;
    if (r != p->rank) {
      base = nullptr;
      if (hipIpcOpenMemHandle(&base, all[size_t(r)], hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
        (void)hipGetLastError();
        ok = 0;
        break;
      }
      p->opened.push_back(base);
    }
    p->peers.data[r] = static_cast<float*>(base);
    p->peers.flags[r] = reinterpret_cast<uint32_t*>(static_cast<char*>(base) + 2 * p->oneshot_cap * 4);
  }
  // every rank must have mapped every peer, or nobody uses the one-shot path
  std::vector<int> oks(size_t(p->world));
  if (!p->rv.allgather(&ok, oks.data(), sizeof(int))) return false;
  for (int v : oks) ok &= v;
  if (!ok) set_pc_err(p, "hipIpcOpenMemHandle failed on some rank: one-shot all-reduce disabled");
  return ok != 0;
}

parallel_context* create_context() {
  auto* p = new parallel_context();
  p->rank = env_int("NAD_TP_RANK", "RANK", "OMPI_COMM_WORLD_RANK", "PMI_RANK", 0);
  p->world = env_int("NAD_TP_SIZE", "WORLD_SIZE", "OMPI_COMM_WORLD_SIZE", "PMI_SIZE", 1);
  p->local_rank = env_int("NAD_TP_LOCAL_RANK", "LOCAL_RANK", "OMPI_COMM_WORLD_LOCAL_RANK", "MPI_LOCALRANKID", p->rank);
  if (p->world < 1 || p->rank < 0 || p->rank >= p->world) {
    set_pc_err(p, "bad rank/world in the environment");
    delete p;
    return nullptr;
  }
  const char* tr = getenv("NAD_PC_TRANSPORT");
  int ndev = 0;
  const bool want_tcp = tr && std::string(tr) == "tcp";
  if (!want_tcp && hipGetDeviceCount(&ndev) == hipSuccess && ndev > 0) {
    p->gpu = true;
    int cur = 0;
    // keep a device the caller already selected (torch.cuda.set_device); otherwise local_rank % devices
    const char* keep = getenv("NAD_PC_KEEP_DEVICE");
    if (keep && atoi(keep)) {
      (void)hipGetDevice(&cur);
    } else {
      cur = p->local_rank % ndev;
      (void)hipSetDevice(cur);
    }
    p->device = cur;
  } else {
    (void)hipGetLastError();
  }
  p->use_rccl = p->gpu && !env_int("NAD_PC_NO_RCCL", nullptr, nullptr, nullptr, 0);
  p->force_rccl = p->use_rccl && env_int("NAD_PC_FORCE_RCCL", nullptr, nullptr, nullptr, 0);
  std::string host = "127.0.0.1";
  int port = env_int("NAD_TP_PORT", nullptr, nullptr, nullptr, 0);
  if (const char* a = getenv("MASTER_ADDR")) host = a;
  if (!port) port = env_int("MASTER_PORT", nullptr, nullptr, nullptr, 29500) + 17;
  if (const char* a = getenv("NAD_TP_ADDR")) {  // host:port
    std::string s(a);
    auto c = s.rfind(':');
    if (c != std::string::npos) {
      host = s.substr(0, c);
      port = atoi(s.c_str() + c + 1);
    }
  }
  p->rv.rank = p->rank;
  p->rv.world = p->world;
  if (!p->rv.open(host, port, env_int("NAD_TP_TIMEOUT", nullptr, nullptr, nullptr, 300))) {
    set_pc_err(p, "rendezvous: " + p->rv.err);
    delete p;
    return nullptr;
  }
  if (p->gpu && (p->world > 1 || p->force_rccl)) {
    p->oneshot = !p->force_rccl && oneshot_init(p);
    if (!rccl_init(p) && p->use_rccl) {
      delete p;
      return nullptr;
    }
  }
  return p;
}

bool is_dev(const void* ptr) {
  hipPointerAttribute_t at;
  if (!ptr || hipPointerGetAttributes(&at, ptr) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return at.type == hipMemoryTypeDevice;
}

float* staging(parallel_context* p, size_t bytes) {
  if (p->stage_bytes < bytes) {
    if (p->stage) (void)hipFree(p->stage);
    p->stage = nullptr;
    p->stage_bytes = 0;
    if (hipMalloc(&p->stage, bytes) != hipSuccess) return nullptr;
    p->stage_bytes = bytes;
  }
  return p->stage;
}

// sum over ranks of host buffers over the rendezvous sockets, in rank order (no GPU)
int tcp_reduce(parallel_context* p, const float* send, float* recv, size_t count) {
  std::vector<float> all(count * size_t(p->world));
  if (!p->rv.allgather(send, all.data(), count * 4)) {
    set_pc_err(p, "tcp reduce: " + p->rv.err);
    return -1;
  }
  for (size_t i = 0; i < count; i++) {
    float s = 0.f;
    for (int r = 0; r < p->world; r++) s += all[size_t(r) * count + i];
    recv[i] = s;
  }
  return 0;
}

int dev_allreduce(parallel_context* p, const float* send, float* recv, size_t count, hipStream_t st) {
  if (p->world == 1 && !p->comm) {
    if (send != recv && hipMemcpyAsync(recv, send, count * 4, hipMemcpyDeviceToDevice, st) != hipSuccess) return -1;
    return 0;
  }
  if (p->oneshot && count <= p->oneshot_cap) {
    const int blocks = int(std::min<size_t>(kOneShotBlocks, (count + 1023) / 1024));
    hipLaunchKernelGGL(nad_oneshot_allreduce_kernel, dim3(std::max(1, blocks)), dim3(kOneShotThreads), 0, st, send,
                       recv, count, p->oneshot_cap, p->rank, p->world, p->peers, p->ctl);
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
  if (!rccl_init(p)) {
    set_pc_err(p, "no RCCL communicator for a message above the one-shot size");
    return -1;
  }
  return ncclAllReduce(send, recv, count, ncclFloat32, ncclSum, p->comm, st) == ncclSuccess ? 0 : -1;
}

}  // namespace

// ------------------------------------------------------------------------------------------------ reference C-ABI
extern "C" parallel_context* init_parallel_context(void) {
  std::lock_guard<std::mutex> lk(g_ctx_mu);
  if (!g_ctx) g_ctx = create_context();
  return g_ctx;
}
extern "C" int get_tp_size(parallel_context* p) { return p ? p->world : 1; }
extern "C" int get_tp_rank(parallel_context* p) { return p ? p->rank : 0; }
extern "C" bool is_master(parallel_context* p) { return !p || p->rank == 0; }

extern "C" void barrier(parallel_context* p) {
  if (!p || p->world == 1) return;
  if (p->gpu) (void)hipDeviceSynchronize();
  char t = 1;
  std::vector<char> all(size_t(p->world));
  if (!p->rv.allgather(&t, all.data(), 1)) set_pc_err(p, "barrier: " + p->rv.err);
}

extern "C" void reduce_add(parallel_context* p, float* send_buffer, float* recv_buffer, size_t count) {
  if (!p) return;
  std::lock_guard<std::mutex> lk(p->mu);
  if (p->world == 1 && !p->comm) {
    if (send_buffer != recv_buffer) {
      if (p->gpu && (is_dev(send_buffer) || is_dev(recv_buffer)))
        (void)hipMemcpyAsync(recv_buffer, send_buffer, count * 4, hipMemcpyDefault, p->stream);
      else
        std::memmove(recv_buffer, send_buffer, count * 4);
    }
    return;
  }
  if (!p->gpu) {
    (void)tcp_reduce(p, send_buffer, recv_buffer, count);
    return;
  }
  const bool ds = is_dev(send_buffer), dr = is_dev(recv_buffer);
  if (ds && dr) {
    if (dev_allreduce(p, send_buffer, recv_buffer, count, p->stream)) set_pc_err(p, "reduce_add failed");
    return;
  }
  // host tensors (ne_layers.c:5466-5476 on CPU tensors): stage, reduce on the device, copy back, synchronous
  float* d = staging(p, count * 4);
  if (!d || hipMemcpyAsync(d, send_buffer, count * 4, hipMemcpyDefault, p->stream) != hipSuccess ||
      dev_allreduce(p, d, d, count, p->stream) ||
      hipMemcpyAsync(recv_buffer, d, count * 4, hipMemcpyDefault, p->stream) != hipSuccess ||
      hipStreamSynchronize(p->stream) != hipSuccess)
    set_pc_err(p, "reduce_add (host buffers) failed");
}

extern "C" void broadcast(parallel_context* p, float* buffer, size_t count) {
  if (!p || p->world == 1) return;
  std::lock_guard<std::mutex> lk(p->mu);
  if (!p->gpu) {
    std::vector<float> all(count * size_t(p->world));
    if (!p->rv.allgather(buffer, all.data(), count * 4)) set_pc_err(p, "broadcast: " + p->rv.err);
    std::memcpy(buffer, all.data(), count * 4);
    return;
  }
  const bool dev = is_dev(buffer);
  float* d = dev ? buffer : staging(p, count * 4);
  if (!rccl_init(p) || !d || (!dev && hipMemcpyAsync(d, buffer, count * 4, hipMemcpyDefault, p->stream)) ||
      ncclBroadcast(d, d, count, ncclFloat32, 0, p->comm, p->stream) != ncclSuccess ||
      (!dev && (hipMemcpyAsync(buffer, d, count * 4, hipMemcpyDefault, p->stream) ||
                hipStreamSynchronize(p->stream))))
    set_pc_err(p, "broadcast failed");
}

// count = elements sent to EACH rank (oneCCL alltoall semantics, parallel_context.cpp:62-64)
extern "C" void alltoall(parallel_context* p, float* send_buffer, float* recv_buffer, size_t count) {
  if (!p) return;
  std::lock_guard<std::mutex> lk(p->mu);
  if (p->world == 1) {  // as reduce_add: device buffers are copied on the context's stream, never by the host
    if (send_buffer != recv_buffer) {
      if (p->gpu && (is_dev(send_buffer) || is_dev(recv_buffer))) {
        if (hipMemcpyAsync(recv_buffer, send_buffer, count * 4, hipMemcpyDefault, p->stream) != hipSuccess)
          set_pc_err(p, "alltoall (world 1) copy failed");
      } else {
        std::memmove(recv_buffer, send_buffer, count * 4);
      }
    }
    return;
  }
  const size_t tot = count * size_t(p->world);
  if (!p->gpu) {
    // rank r receives block r of every rank's send buffer
    std::vector<float> all(tot * size_t(p->world));
    if (!p->rv.allgather(send_buffer, all.data(), tot * 4)) {
      set_pc_err(p, "alltoall: " + p->rv.err);
      return;
    }
    for (int s = 0; s < p->world; s++)
      std::memcpy(recv_buffer + size_t(s) * count, all.data() + size_t(s) * tot + size_t(p->rank) * count, count * 4);
    return;
  }
  const bool ds = is_dev(send_buffer), dr = is_dev(recv_buffer);
  float* d = (ds && dr) ? nullptr : staging(p, 2 * tot * 4);
  const float* s = ds ? send_buffer : d;
  float* r = dr ? recv_buffer : (d ? d + tot : nullptr);
  if (!rccl_init(p) || (!ds && (!d || hipMemcpyAsync(d, send_buffer, tot * 4, hipMemcpyDefault, p->stream))) ||
      ncclAllToAll(s, r, count, ncclFloat32, p->comm, p->stream) != ncclSuccess ||
      (!dr && (hipMemcpyAsync(recv_buffer, r, tot * 4, hipMemcpyDefault, p->stream) ||
               hipStreamSynchronize(p->stream))))
    set_pc_err(p, "alltoall failed");
}

// ------------------------------------------------------------------------------------------------ native extensions
extern "C" int nad_pc_allreduce_f32(parallel_context* p, const float* send, float* recv, size_t count, void* stream) {
  if (!p) return -1;
  std::lock_guard<std::mutex> lk(p->mu);
  if (!p->gpu) return tcp_reduce(p, send, recv, count);
  return dev_allreduce(p, send, recv, count, static_cast<hipStream_t>(stream));
}

extern "C" int nad_pc_set_stream(parallel_context* p, void* stream) {
  if (!p) return -1;
  p->stream = static_cast<hipStream_t>(stream);
  return 0;
}

extern "C" double nad_pc_max_f64(parallel_context* p, double v) {
  if (!p || p->world == 1) return v;
  std::vector<double> all(size_t(p->world));
  if (!p->rv.allgather(&v, all.data(), sizeof(double))) {
    set_pc_err(p, "max: " + p->rv.err);
    return v;
  }
  return *std::max_element(all.begin(), all.end());
}

// 0 ok; 1 a one-shot all-reduce gave up waiting for a peer (synchronous); -1 no context
extern "C" int nad_pc_status(parallel_context* p) {
  if (!p) return -1;
  if (!p->ctl) return 0;
  uint32_t c[3] = {0, 0, 0};
  if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(c, p->ctl, sizeof(c), hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  return int(c[2]);
}

// bit 0: GPU transport, bit 1: one-shot IPC all-reduce available, bit 2: RCCL communicator up, bit 3: the one-shot
// buffer is uncached fine-grained memory (hipExtMallocWithFlags(hipDeviceMallocUncached)), not the hipMalloc fallback
extern "C" int nad_pc_info(parallel_context* p) {
  if (!p) return -1;
  return (p->gpu ? 1 : 0) | (p->oneshot ? 2 : 0) | (p->comm ? 4 : 0) | (p->oneshot && p->oneshot_uncached ? 8 : 0);
}

extern "C" const char* nad_pc_last_error(parallel_context* p) { return p ? p->err.c_str() : "no parallel context"; }

extern "C" void nad_pc_destroy(parallel_context* p) {
  std::lock_guard<std::mutex> lk(g_ctx_mu);
  if (!p) return;
  if (p->gpu) (void)hipDeviceSynchronize();
  if (p->world > 1) {  // nobody unmaps a peer buffer while another rank may still read it
    char t = 1;
    std::vector<char> all(size_t(p->world));
    (void)p->rv.allgather(&t, all.data(), 1);
  }
  if (p->comm) (void)ncclCommDestroy(p->comm);
  for (void* b : p->opened) (void)hipIpcCloseMemHandle(b);
  if (p->own) (void)hipFree(p->own);
  if (p->ctl) (void)hipFree(p->ctl);
  if (p->stage) (void)hipFree(p->stage);
  p->rv.close_all();
  if (p == g_ctx) g_ctx = nullptr;
  delete p;
}
