// pkc_dp.hip — chunk-level data parallelism for non-Python hosts (SURVEY §8b "pkc_dp_allreduce",
// §8e): the one exchange of the training step, an RCCL all-reduce (SUM) of the flat fp32 gradient
// buffer over xGMI.  The Python host (pkc.dist) uses torch.distributed's RCCL communicator; these
// entry points let a C / C++ / cgo host run the same step: rank 0 makes an id, ships its 128 bytes
// to the other ranks by any channel, every rank creates its communicator on its own GPU, then
// calls pkc_dp_allreduce between the backward and the optimizer launches on its step stream.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include "pkc_common.h"

namespace {
int rccl_status(ncclResult_t r, const char* where) {
  if (r == ncclSuccess) return PKC_OK;
  pkc::set_error("%s: %s", where, ncclGetErrorString(r));
  return PKC_ERR_HIP;
}
}  // namespace

extern "C" int pkc_dp_unique_id_bytes(void) { return NCCL_UNIQUE_ID_BYTES; }

extern "C" int pkc_dp_unique_id(void* id_out) {
  PKC_CHECK_ARG(id_out, "pkc_dp_unique_id: null output");
  ncclUniqueId id;
  const int st = rccl_status(ncclGetUniqueId(&id), "pkc_dp_unique_id");
  if (st == PKC_OK) memcpy(id_out, &id, sizeof(id));
  return st;
}

extern "C" int pkc_dp_comm_init(void** comm_out, int world, const void* id, int rank, int device) {
  PKC_CHECK_ARG(comm_out && id && world >= 1 && rank >= 0 && rank < world,
                "pkc_dp_comm_init: bad arguments (world %d rank %d)", world, rank);
  if (device >= 0 && hipSetDevice(device) != hipSuccess) {
    pkc::set_error("pkc_dp_comm_init: hipSetDevice(%d) failed", device);
    return PKC_ERR_HIP;
  }
  ncclUniqueId uid;
  memcpy(&uid, id, sizeof(uid));
  ncclComm_t c = nullptr;
  const int st = rccl_status(ncclCommInitRank(&c, world, uid, rank), "pkc_dp_comm_init");
  *comm_out = st == PKC_OK ? reinterpret_cast<void*>(c) : nullptr;
  return st;
}

extern "C" int pkc_dp_allreduce(void* comm, float* buf, int64_t n, void* stream) {
  PKC_CHECK_ARG(comm && (buf || n == 0) && n >= 0, "pkc_dp_allreduce: bad arguments");
  if (n == 0) return PKC_OK;
  return rccl_status(ncclAllReduce(buf, buf, (size_t)n, ncclFloat32, ncclSum,
                                   reinterpret_cast<ncclComm_t>(comm), pkc::S(stream)),
                     "pkc_dp_allreduce");
}

extern "C" int pkc_dp_comm_destroy(void* comm) {
  if (!comm) return PKC_OK;
  return rccl_status(ncclCommDestroy(reinterpret_cast<ncclComm_t>(comm)), "pkc_dp_comm_destroy");
}
