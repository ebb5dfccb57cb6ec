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
// Linked against the librccl.so that torch itself loads, so the process holds one RCCL.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <rccl/rccl.h>

#include <string>
#include <vector>

namespace {

std::vector<ncclComm_t> g_comms;   // handle = index (destroyed slots hold nullptr)

void rccl_check(ncclResult_t r, const char* what) {
  TORCH_CHECK(r == ncclSuccess, "RCCL ", what, " failed: ", ncclGetErrorString(r));
}

ncclComm_t comm_of(int64_t h) {
  TORCH_CHECK(h >= 0 && h < (int64_t)g_comms.size() && g_comms[h] != nullptr, "invalid RCCL communicator handle");
  return g_comms[h];
}

}  // namespace

// a fresh unique id (rank 0), as bytes for the process-group broadcast
pybind11::bytes comm_unique_id() {
  ncclUniqueId id;
  rccl_check(ncclGetUniqueId(&id), "ncclGetUniqueId");
  return pybind11::bytes(reinterpret_cast<const char*>(&id), sizeof(id));
}

// collective over all ranks (each passes the same id): returns the handle
int64_t comm_init(const std::string& id_bytes, int64_t nranks, int64_t rank) {
  TORCH_CHECK(id_bytes.size() == sizeof(ncclUniqueId), "ncclUniqueId must be ", sizeof(ncclUniqueId), " bytes");
  TORCH_CHECK(nranks >= 1 && rank >= 0 && rank < nranks, "rank / nranks");
  ncclUniqueId id;
  memcpy(&id, id_bytes.data(), sizeof(id));
  ncclComm_t c = nullptr;
  rccl_check(ncclCommInitRank(&c, (int)nranks, id, (int)rank), "ncclCommInitRank");
  g_comms.push_back(c);
  return (int64_t)g_comms.size() - 1;
}

// in-place sum (mean: average) of a contiguous fp32 / fp64 device tensor over the communicator,
// enqueued on `stream` (0: the current torch stream)
void comm_allreduce(int64_t h, torch::Tensor t, bool mean, int64_t stream) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous() && (t.scalar_type() == at::kFloat || t.scalar_type() == at::kDouble),
              "fp32 / fp64 contiguous device tensor");
  const hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : at::hip::getCurrentHIPStream().stream();
  const ncclDataType_t ty = t.scalar_type() == at::kFloat ? ncclFloat : ncclDouble;
  rccl_check(ncclAllReduce(t.data_ptr(), t.data_ptr(), (size_t)t.numel(), ty, mean ? ncclAvg : ncclSum, comm_of(h), s),
             "ncclAllReduce");
}

void comm_destroy(int64_t h) {
  ncclComm_t c = comm_of(h);
  rccl_check(ncclCommDestroy(c), "ncclCommDestroy");
  g_comms[h] = nullptr;
}

void register_comm(pybind11::module& m) {
  m.def("comm_unique_id", &comm_unique_id);
  m.def("comm_init", &comm_init);
  m.def("comm_allreduce", &comm_allreduce, pybind11::arg("handle"), pybind11::arg("t"), pybind11::arg("mean") = false,
        pybind11::arg("stream") = 0);
  m.def("comm_destroy", &comm_destroy);
}
