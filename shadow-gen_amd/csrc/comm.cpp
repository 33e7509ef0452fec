// comm.cpp — round-edge exchange between shards over RCCL (xGMI on one MI355X node).
//
// The reference has no distributed backend: cross-host packet pushes are
// Mutex<EventQueue> pushes between threads (core/worker.rs:603-613) and the round minimum
// is a per-thread reduction (core/manager.rs:623-628). With hosts sharded over GPUs, the
// same two steps become, per round and entirely stream-ordered (no host round trip):
//   1. grouped ncclSend/ncclRecv of each peer's fixed-size event slot + its count,
//   2. k_import files received events into the local calendar,
//   3. k_finalize(local) computes {min next event, min used latency} for this shard,
//   4. ncclAllReduce(min, uint64, 2) in place, then k_advance moves the window.
// Every produced event has time >= the window end (worker.rs:386-390), so nothing needs
// to cross shards inside a round.

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>

#include "sgn_internal.h"

namespace sgn {
void launch_finalize_local(sgn_ctx* ctx);
void launch_import(sgn_ctx* ctx);
void launch_advance(sgn_ctx* ctx, const uint64_t* red);
}  // namespace sgn

using namespace sgn;

static_assert(sizeof(ncclUniqueId) <= SGN_COMM_ID_BYTES, "ncclUniqueId size");

namespace sgn {
void comm_destroy(sgn_ctx* ctx) {
  if (ctx && ctx->comm) {
    ncclCommDestroy((ncclComm_t)ctx->comm);
    ctx->comm = nullptr;
  }
}
}  // namespace sgn

extern "C" {

int sgn_comm_get_unique_id(uint8_t id_out[SGN_COMM_ID_BYTES]) {
  if (!id_out) return SGN_EINVAL;
  ncclUniqueId u;
  if (ncclGetUniqueId(&u) != ncclSuccess) return SGN_EDEVICE;
  std::memset(id_out, 0, SGN_COMM_ID_BYTES);
  std::memcpy(id_out, &u, sizeof(u));
  return 0;
}

int sgn_comm_init(sgn_ctx* ctx, const uint8_t id[SGN_COMM_ID_BYTES], uint64_t slot_events) {
  if (!ctx || !id) return SGN_EINVAL;
  if (ctx->nranks < 2) return set_error(ctx, SGN_ESTATE, "sgn_comm_init needs shard_count >= 2");
  if (slot_events == 0 || slot_events > (1ULL << 26))
    return set_error(ctx, SGN_EINVAL, "exchange_slot_events must be in [1, 2^26]");
  SGN_HIP(ctx, hipSetDevice(ctx->device));
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  ncclComm_t comm;
  ncclResult_t r = ncclCommInitRank(&comm, (int)ctx->nranks, u, (int)ctx->rank);
  if (r != ncclSuccess)
    return set_error(ctx, SGN_EDEVICE, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
  comm_destroy(ctx);
  ctx->comm = comm;
  ctx->xslot = slot_events;
  return 0;
}

}  // extern "C"

namespace sgn {
int comm_round_exchange(sgn_ctx* ctx) {
  DevSim& S = ctx->S;
  ncclComm_t comm = (ncclComm_t)ctx->comm;
  hipStream_t st = ctx->stream;
  const size_t slot_bytes = (size_t)S.xslot * sizeof(EvRec);
  ncclResult_t r = ncclGroupStart();
  for (uint32_t p = 0; p < S.n_ranks && r == ncclSuccess; p++) {
    if (p == S.rank) continue;
    r = ncclSend(S.xout + (size_t)p * S.xslot, slot_bytes, ncclUint8, (int)p, comm, st);
    if (r == ncclSuccess)
      r = ncclRecv(S.xin + (size_t)p * S.xslot, slot_bytes, ncclUint8, (int)p, comm, st);
    if (r == ncclSuccess) r = ncclSend(S.xout_n + p, 1, ncclUint32, (int)p, comm, st);
    if (r == ncclSuccess) r = ncclRecv(S.xin_n + p, 1, ncclUint32, (int)p, comm, st);
  }
  ncclResult_t r2 = ncclGroupEnd();
  if (r != ncclSuccess || r2 != ncclSuccess)
    return set_error(ctx, SGN_EDEVICE, std::string("RCCL exchange: ") +
                                           ncclGetErrorString(r != ncclSuccess ? r : r2));
  SGN_HIP(ctx, hipMemsetAsync(S.xin_n + S.rank, 0, 4, st));
  launch_import(ctx);
  SGN_HIP(ctx, hipMemsetAsync(S.xout_n, 0, (size_t)S.n_ranks * 4, st));
  launch_finalize_local(ctx);
  // {round_min, min_used} are adjacent u64 fields of Ctrl: reduce both in place
  uint64_t* red = &S.ctrl->round_min;
  r = ncclAllReduce(red, red, 2, ncclUint64, ncclMin, comm, st);
  if (r != ncclSuccess)
    return set_error(ctx, SGN_EDEVICE, std::string("RCCL all-reduce: ") + ncclGetErrorString(r));
  launch_advance(ctx, red);
  return 0;
}

}  // namespace sgn
