// hq_comm.hip — the one collective of the sharded search: an RCCL all-gather of
// every rank's per-shard top-k records over xGMI, behind the C-ABI so a non-Python host can run the
// sharded search (cfg4) without torch.distributed.
//
// The reference has no collective: its closest analogue is the per-video thread fan-out whose result
// lists are concatenated and re-sorted (core/video_search.py:722-875).  Here each rank contributes a
// fixed-size record block (hq_mi355x.distributed: Q x (M + 1) x (2 + W) float64, ~1.3 MB per rank at
// Q = 1000, M = 20), so the exchange is one ncclAllGather: latency-bound, far below the 7 x 153 GB/s
// xGMI budget, and the merge (hq_progressive_final) runs on every rank.
//
// Communicator bootstrap: rank 0 calls hq_comm_unique_id, the 128 id bytes travel to the other ranks
// by any out-of-band channel (a TCP store, a file, MPI), and every rank calls hq_comm_init_rank on its
// own device (the current HIP device).  RCCL returns its own error strings (ncclGetErrorString).
#include "hq_common.h"

#include <rccl/rccl.h>
#include <string.h>

namespace hq {

#define HQ_CHECK_NCCL(expr)                                                                          \
  do {                                                                                               \
    ncclResult_t _r = (expr);                                                                        \
    if (_r != ncclSuccess) return ::hq::fail(HQ_E_HIP, "%s failed: %s", #expr, ncclGetErrorString(_r)); \
  } while (0)

static_assert(sizeof(ncclUniqueId) == HQ_COMM_ID_BYTES, "RCCL unique id size");

}  // namespace hq

using namespace hq;

extern "C" {

int hq_comm_unique_id(void* id_out) {
  if (!id_out) return fail(HQ_E_INVALID, "null buffer");
  ncclUniqueId id;
  HQ_CHECK_NCCL(ncclGetUniqueId(&id));
  memcpy(id_out, &id, sizeof(id));
  return HQ_OK;
}

int hq_comm_init_rank(void** comm, int nranks, const void* id, int rank) {
  if (!comm || !id) return fail(HQ_E_INVALID, "null buffer");
  if (nranks < 1 || rank < 0 || rank >= nranks) return fail(HQ_E_INVALID, "rank %d of %d", rank, nranks);
  ncclUniqueId uid;
  memcpy(&uid, id, sizeof(uid));
  ncclComm_t c = nullptr;
  HQ_CHECK_NCCL(ncclCommInitRank(&c, nranks, uid, rank));
  *comm = (void*)c;
  return HQ_OK;
}

int hq_comm_destroy(void* comm) {
  if (!comm) return HQ_OK;
  HQ_CHECK_NCCL(ncclCommDestroy((ncclComm_t)comm));
  return HQ_OK;
}

int hq_comm_size(void* comm, int* nranks, int* rank) {
  if (!comm) return fail(HQ_E_INVALID, "null communicator");
  if (nranks) HQ_CHECK_NCCL(ncclCommCount((ncclComm_t)comm, nranks));
  if (rank) HQ_CHECK_NCCL(ncclCommUserRank((ncclComm_t)comm, rank));
  return HQ_OK;
}

int hq_allgather_topk(void* comm, const void* send, void* recv, size_t bytes, hq_stream_t stream) {
  if (!comm) return fail(HQ_E_INVALID, "null communicator");
  if (bytes == 0) return HQ_OK;
  if (!send || !recv) return fail(HQ_E_INVALID, "null buffer");
  // bytes as ncclUint8: the records are opaque to the collective (every rank sends the same size)
  HQ_CHECK_NCCL(ncclAllGather(send, recv, bytes, ncclUint8, (ncclComm_t)comm, (hipStream_t)stream));
  return HQ_OK;
}

}  // extern "C"
