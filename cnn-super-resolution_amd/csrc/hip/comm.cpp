// comm.cpp -- the RCCL gradient-reduction stage of srcnn.h.
//
// The reference trains on one OpenCL queue (src/Main_cl.cpp:157-195:
// execute_batch over the whole training set, then update_parameters); it has
// no multi-device path.  Data-parallel training here shards the tile batch
// over devices: every device accumulates the gradients of its shard into the
// flat [gW1|gB1|gW2|gB2|gW3|gB3] buffer, ONE in-place all-reduce(SUM) over
// xGMI combines them, and every device applies the same srcnn_update_all with
// batch = the global tile count, so the parameter replicas stay identical.
//
// Two ways to build communicators, both plain RCCL:
//   one process per GPU  : srcnn_comm_id on one rank, the 128-byte id shipped
//                          to the others by the caller, srcnn_comm_init_rank
//   one process, N GPUs  : srcnn_comm_init_all (ncclCommInitAll); each device
//                          then driven by its own host thread
// The collective is enqueued on the caller's compute stream, so it is ordered
// after the gradient kernels and before the update without host syncs.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstring>

#include "common.hpp"

#define SRCNN_NCCL_TRY(expr)                                                             \
  do {                                                                                   \
    ncclResult_t r_ = (expr);                                                            \
    if (r_ != ncclSuccess)                                                               \
      return ::srcnn::fail(SRCNN_ERR_COMM, "%s failed: %s", #expr, ncclGetErrorString(r_)); \
  } while (0)

static_assert(sizeof(ncclUniqueId) == SRCNN_COMM_ID_BYTES, "RCCL unique id size");

extern "C" {

int srcnn_comm_id(uint8_t* id) {
  SRCNN_REQUIRE(id, "srcnn_comm_id: null id buffer");
  ncclUniqueId u;
  SRCNN_NCCL_TRY(ncclGetUniqueId(&u));
  std::memcpy(id, &u, sizeof(u));
  return SRCNN_OK;
}

int srcnn_comm_init_rank(srcnn_comm_t* comm, int nranks, const uint8_t* id, int rank) {
  SRCNN_REQUIRE(comm && id, "srcnn_comm_init_rank: null argument");
  SRCNN_REQUIRE(nranks > 0 && rank >= 0 && rank < nranks,
                "srcnn_comm_init_rank: rank %d out of [0, %d)", rank, nranks);
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  ncclComm_t c = nullptr;
  SRCNN_NCCL_TRY(ncclCommInitRank(&c, nranks, u, rank));
  *comm = c;
  return SRCNN_OK;
}

int srcnn_comm_init_all(srcnn_comm_t* comms, int ndev, const int* devices) {
  SRCNN_REQUIRE(comms && ndev > 0, "srcnn_comm_init_all: need an output array and ndev > 0");
  int n = 0;
  SRCNN_HIP_TRY(hipGetDeviceCount(&n));
  for (int i = 0; devices && i < ndev; i++)
    SRCNN_REQUIRE(devices[i] >= 0 && devices[i] < n, "srcnn_comm_init_all: device %d out of [0, %d)",
                  devices[i], n);
  SRCNN_REQUIRE(devices || ndev <= n, "srcnn_comm_init_all: %d devices requested, %d present", ndev, n);
  int cur = 0;
  SRCNN_HIP_TRY(hipGetDevice(&cur));
  ncclComm_t* c = reinterpret_cast<ncclComm_t*>(comms);
  ncclResult_t r = ncclCommInitAll(c, ndev, devices);
  (void)hipSetDevice(cur);  // ncclCommInitAll walks the devices
  if (r != ncclSuccess)
    return srcnn::fail(SRCNN_ERR_COMM, "ncclCommInitAll(%d) failed: %s", ndev, ncclGetErrorString(r));
  return SRCNN_OK;
}

int srcnn_comm_destroy(srcnn_comm_t comm) {
  if (comm) SRCNN_NCCL_TRY(ncclCommDestroy(reinterpret_cast<ncclComm_t>(comm)));
  return SRCNN_OK;
}

int srcnn_comm_rank(srcnn_comm_t comm, int* rank, int* nranks) {
  SRCNN_REQUIRE(comm, "srcnn_comm_rank: null communicator");
  ncclComm_t c = reinterpret_cast<ncclComm_t>(comm);
  if (rank) SRCNN_NCCL_TRY(ncclCommUserRank(c, rank));
  if (nranks) SRCNN_NCCL_TRY(ncclCommCount(c, nranks));
  return SRCNN_OK;
}

int srcnn_comm_group_start(void) {
  SRCNN_NCCL_TRY(ncclGroupStart());
  return SRCNN_OK;
}

int srcnn_comm_group_end(void) {
  SRCNN_NCCL_TRY(ncclGroupEnd());
  return SRCNN_OK;
}

int srcnn_comm_version(int* version, char* path, size_t len) {
  if (version) SRCNN_NCCL_TRY(ncclGetVersion(version));
  if (path && len) {
    // the file the dynamic loader bound ncclAllReduce to (its DT_NEEDED
    // soname librccl.so.1 resolves to whichever copy loaded first)
    Dl_info di;
    const void* fn = reinterpret_cast<const void*>(&ncclAllReduce);
    if (dladdr(fn, &di) && di.dli_fname)
      std::snprintf(path, len, "%s", di.dli_fname);
    else
      path[0] = 0;
  }
  return SRCNN_OK;
}

int srcnn_allreduce_grads(srcnn_comm_t comm, float* buf, size_t count, srcnn_stream_t stream) {
  SRCNN_REQUIRE(comm, "srcnn_allreduce_grads: null communicator");
  if (count == 0) return SRCNN_OK;
  SRCNN_REQUIRE(buf, "srcnn_allreduce_grads: null buffer");
  SRCNN_PROFILE("allreduce_grads", srcnn::as_stream(stream));
  SRCNN_NCCL_TRY(ncclAllReduce(buf, buf, count, ncclFloat32, ncclSum,
                               reinterpret_cast<ncclComm_t>(comm), srcnn::as_stream(stream)));
  return SRCNN_OK;
}

}  // extern "C"
