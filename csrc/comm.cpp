// Native RCCL communicator for the gradient all-reduce of the DPPO workers (the reference's chief
// gradient sum, chief.py:13-20 / train.py:169-175, as one collective over xGMI).
//
// torch.distributed's ProcessGroupNCCL runs every collective on its own internal stream, so each
// all-reduce costs two cross-stream event hops (compute -> RCCL stream -> compute), each a
// barrier packet the compute queue idles on: ~26 us of GPU idle per hop pair measured at world
// size 1 (profiles/r3/rccl_forced_vs_plain.md).  This communicator is created once per worker
// from an ncclUniqueId that rank 0 broadcasts over the existing process group, and launches the
// all-reduce on the stream the caller names — the compute stream itself (in stream order: no
// event hops at all) or a side stream the caller fences with its own events.
//
// Failure detection (the reference deadlocks forever on a dead worker, chief.py:13,
// Q21).  Because these collectives bypass ProcessGroupNCCL, they also bypass its watchdog, so the
// communicator carries its own:
//   * the communicator is NON-BLOCKING (ncclConfig_t.blocking = 0): ncclCommInitRank returns at
//     once and comm_init polls ncclCommGetAsyncError with a deadline — a rank that never joins
//     turns into an exception (after ncclCommAbort) on every other rank instead of a hang;
//   * an enqueue that reports ncclInProgress (lazy connection setup) is polled the same way;
//   * comm_status exposes ncclCommGetAsyncError so the host-side wait loops
//     (parallel/dist.py DistContext.wait_event) can stop at the first asynchronous error;
//   * comm_abort calls ncclCommAbort: the RCCL kernels poll the abort flag and exit, so a
//     collective stuck on a dead peer drains from the GPU before the process exits (a kernel
//     whose waves never finish must not outlive its process).
//
// Linked against the librccl.so that torch itself loads, so the process holds one RCCL.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <rccl/rccl.h>

#include <chrono>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace {

struct Comm {
  ncclComm_t comm = nullptr;   // nullptr once destroyed / aborted
  double timeout_s = 300.0;
};

// handle = index.  g_mu guards every slot's comm pointer: the heartbeat thread may abort a
// communicator (comm_abort) while the main thread polls it with the GIL released (wait_ready)
std::mutex g_mu;
std::vector<std::unique_ptr<Comm>> g_comms;

void rccl_check(ncclResult_t r, const char* what) {
  TORCH_CHECK(r == ncclSuccess, "RCCL ", what, " failed: ", ncclGetErrorString(r));
}

Comm& comm_of(int64_t h) {
  std::lock_guard<std::mutex> lk(g_mu);
  TORCH_CHECK(h >= 0 && h < (int64_t)g_comms.size() && g_comms[h]->comm != nullptr,
              "invalid (destroyed or aborted) RCCL communicator handle");
  return *g_comms[h];
}

// poll a non-blocking communicator (the slot's, or `raw` before a slot exists) until its pending
// operation leaves ncclInProgress; the GIL is released while waiting (the peers' progress never
// depends on this process's Python thread).  Returns the final state: ncclInProgress means
// timeout_s passed, ncclInvalidUsage that another thread aborted the communicator meanwhile.
ncclResult_t wait_ready(Comm* slot, ncclComm_t raw, double timeout_s) {
  ncclResult_t st = ncclInProgress;
  pybind11::gil_scoped_release nogil;
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    {
      std::lock_guard<std::mutex> lk(g_mu);
      ncclComm_t c = slot != nullptr ? slot->comm : raw;
      if (c == nullptr) return ncclInvalidUsage;
      if (ncclCommGetAsyncError(c, &st) != ncclSuccess) st = ncclInternalError;
    }
    if (st != ncclInProgress) break;
    const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (el > timeout_s) break;
    std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
  return st;
}

// an operation that failed (or timed out): abort the communicator (its RCCL kernels exit), clear
// the slot (null slot: comm_init, before the slot exists) and throw
[[noreturn]] void fail(Comm* slot, ncclComm_t raw, ncclResult_t st, double timeout_s, const char* what) {
  {
    std::lock_guard<std::mutex> lk(g_mu);
    ncclComm_t c = slot != nullptr ? slot->comm : raw;
    if (slot != nullptr) slot->comm = nullptr;
    if (c != nullptr) ncclCommAbort(c);
  }
  const std::string why = st == ncclInProgress ? "timed out after " + std::to_string(timeout_s) + " s"
                          : st == ncclInvalidUsage ? std::string("aborted by another thread")
                                                   : std::string("failed: ") + ncclGetErrorString(st);
  TORCH_CHECK(false, "RCCL ", what, " ", why, "; communicator aborted");
  throw;   // unreachable (TORCH_CHECK(false) throws)
}

}  // namespace

// a fresh unique id (rank 0), as bytes for the process-group broadcast
pybind11::bytes comm_unique_id() {
  ncclUniqueId id;
  rccl_check(ncclGetUniqueId(&id), "ncclGetUniqueId");
  return pybind11::bytes(reinterpret_cast<const char*>(&id), sizeof(id));
}

// collective over all ranks (each passes the same id): returns the handle.  Bounded: a peer that
// never joins makes this throw after timeout_s (the half-built communicator is aborted).
int64_t comm_init(const std::string& id_bytes, int64_t nranks, int64_t rank, double timeout_s) {
  TORCH_CHECK(id_bytes.size() == sizeof(ncclUniqueId), "ncclUniqueId must be ", sizeof(ncclUniqueId), " bytes");
  TORCH_CHECK(nranks >= 1 && rank >= 0 && rank < nranks, "rank / nranks");
  TORCH_CHECK(timeout_s > 0, "timeout_s > 0");
  ncclUniqueId id;
  memcpy(&id, id_bytes.data(), sizeof(id));
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;
  ncclComm_t c = nullptr;
  const ncclResult_t r = ncclCommInitRankConfig(&c, (int)nranks, id, (int)rank, &cfg);
  if (r != ncclSuccess && r != ncclInProgress) {
    if (c != nullptr) ncclCommAbort(c);
    rccl_check(r, "ncclCommInitRankConfig");
  }
  const ncclResult_t st = wait_ready(nullptr, c, timeout_s);
  if (st != ncclSuccess) fail(nullptr, c, st, timeout_s, "ncclCommInitRankConfig");
  std::lock_guard<std::mutex> lk(g_mu);
  g_comms.push_back(std::make_unique<Comm>(Comm{c, timeout_s}));
  return (int64_t)g_comms.size() - 1;
}

// in-place sum (mean: average) of a contiguous fp32 / fp64 device tensor over the communicator,
// enqueued on `stream` (0: the current torch stream)
void comm_allreduce(int64_t h, torch::Tensor t, bool mean, int64_t stream) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous() && (t.scalar_type() == at::kFloat || t.scalar_type() == at::kDouble),
              "fp32 / fp64 contiguous device tensor");
  Comm& c = comm_of(h);
  const hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : at::hip::getCurrentHIPStream().stream();
  const ncclDataType_t ty = t.scalar_type() == at::kFloat ? ncclFloat : ncclDouble;
  const ncclResult_t r = ncclAllReduce(t.data_ptr(), t.data_ptr(), (size_t)t.numel(), ty, mean ? ncclAvg : ncclSum,
                                       c.comm, s);
  // ncclInProgress: the enqueue is finishing asynchronously (e.g. first-use connection setup)
  const ncclResult_t st = r == ncclInProgress ? wait_ready(&c, nullptr, c.timeout_s) : r;
  if (st != ncclSuccess) fail(&c, nullptr, st, c.timeout_s, "ncclAllReduce");
}

// ncclCommGetAsyncError of the communicator: 0 (ncclSuccess), 7 (ncclInProgress) or an error
// code; -1 for a destroyed / aborted handle
int64_t comm_status(int64_t h) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (h < 0 || h >= (int64_t)g_comms.size() || g_comms[h]->comm == nullptr) return -1;
  ncclResult_t st = ncclSuccess;
  if (ncclCommGetAsyncError(g_comms[h]->comm, &st) != ncclSuccess) return (int64_t)ncclInternalError;
  return (int64_t)st;
}

// ncclCommAbort: every RCCL kernel of the communicator exits (no completion), the handle is dead.
// Safe from any thread (the heartbeat's dead-peer path calls it while the main thread waits).
void comm_abort(int64_t h) {
  pybind11::gil_scoped_release nogil;
  std::lock_guard<std::mutex> lk(g_mu);
  if (h < 0 || h >= (int64_t)g_comms.size() || g_comms[h]->comm == nullptr) return;
  ncclComm_t c = g_comms[h]->comm;
  g_comms[h]->comm = nullptr;
  ncclCommAbort(c);
}

void comm_destroy(int64_t h) {
  Comm& c = comm_of(h);
  const ncclResult_t r = ncclCommFinalize(c.comm);
  const ncclResult_t st = r == ncclInProgress ? wait_ready(&c, nullptr, c.timeout_s) : r;
  if (st != ncclSuccess) fail(&c, nullptr, st, c.timeout_s, "ncclCommFinalize");
  ncclComm_t comm;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    comm = c.comm;
    c.comm = nullptr;
  }
  if (comm != nullptr) rccl_check(ncclCommDestroy(comm), "ncclCommDestroy");
}

void register_comm(pybind11::module& m) {
  m.def("comm_unique_id", &comm_unique_id);
  m.def("comm_init", &comm_init, pybind11::arg("id"), pybind11::arg("nranks"), pybind11::arg("rank"),
        pybind11::arg("timeout_s") = 300.0);
  m.def("comm_allreduce", &comm_allreduce, pybind11::arg("handle"), pybind11::arg("t"), pybind11::arg("mean") = false,
        pybind11::arg("stream") = 0);
  m.def("comm_status", &comm_status);
  m.def("comm_abort", &comm_abort);
  m.def("comm_destroy", &comm_destroy);
}
