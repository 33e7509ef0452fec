// comm.cpp — round-edge exchange between shards over RCCL (xGMI on one MI355X node).
//
// The reference has no distributed backend: cross-host packet pushes are
// Mutex<EventQueue> pushes between threads (core/worker.rs:603-613) and the round minimum
// is a per-thread reduction (core/manager.rs:623-628). With hosts sharded over GPUs, the
// same two steps become, per round and entirely stream-ordered (no host round trip):
//   1. k_execute's last wave does the local round edge (bucket bookkeeping) and writes one
//      32-byte message per peer: {runs sent to it, this shard's min next event including
//      the runs it exported, its min used latency},
//   2. ONE grouped ncclSend/ncclRecv moves each peer's fixed-size run slot and message,
//   3. k_import files the received runs into the local calendar, and its last block
//      reduces the n messages (the global min: what an all-reduce would give) and moves
//      the window — every shard computes the same window.
// Every produced event has time >= the window end (worker.rs:386-390), so nothing needs
// to cross shards inside a round.

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "sgn_internal.h"

namespace sgn {
void launch_execute(sgn_ctx* ctx);
void launch_import(sgn_ctx* ctx);
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
int ctrl_sync(sgn_ctx* ctx);  // engine.hip: the control block to the host, overflow check
int resolve_pools(sgn_ctx* ctx);  // engine.hip: a held round edge's pool growth
int grow_exchange_slot(sgn_ctx* ctx);  // engine.hip: larger exchange slots (runs past a slot)

uint64_t comm_round_bytes(const sgn_ctx* ctx) {
  return ctx->nranks > 1 && ctx->comm ? (uint64_t)(ctx->nranks - 1) * ((uint64_t)(XHDR + ctx->xsz_cur) * sizeof(EvRec)) : 0;
}

// ONE grouped send/recv: per peer one message of the 32-byte round-edge record and the first
// sz runs of its slot (one send and one receive per peer)
static int exchange(sgn_ctx* ctx, uint32_t sz) {
  DevSim& S = ctx->S;
  ncclComm_t comm = (ncclComm_t)ctx->comm;
  hipStream_t st = ctx->stream;
  // a peer's block: the message (one 32-byte record), then the runs
  const size_t bytes = (size_t)(XHDR + sz) * sizeof(EvRec);
  const size_t blk = (size_t)S.xslot + XHDR;
  ncclResult_t r = ncclGroupStart();
  for (uint32_t p = 0; p < S.n_ranks && r == ncclSuccess; p++) {
    if (p == S.rank) continue;
    r = ncclSend(S.xout + p * blk, bytes, ncclUint8, (int)p, comm, st);
    if (r == ncclSuccess) r = ncclRecv(S.xin + p * blk, bytes, ncclUint8, (int)p, comm, st);
  }
  ncclResult_t r2 = ncclGroupEnd();
  if (r != ncclSuccess || r2 != ncclSuccess)
    return set_error(ctx, SGN_EDEVICE, std::string("RCCL exchange: ") +
                                           ncclGetErrorString(r != ncclSuccess ? r : r2));
  return 0;
}

int comm_round_exchange(sgn_ctx* ctx) {
  // k_execute's last wave has already done the local round edge and written this shard's
  // message for every peer (run count, local min next event incl. exported runs, local min
  // used latency, its largest per-peer count): ONE grouped send/recv moves the first
  // xsz_cur runs of every slot and the messages, then one kernel on every shard imports the
  // runs and reduces the messages (no all-reduce, no memsets). xsz_cur follows the largest
  // per-peer count seen (x2, a power of two), so a round moves about what it produced
  // instead of the whole slot.
  if (int rc = exchange(ctx, ctx->xsz_cur)) return rc;
  if (!ctx->capturing) ctx->x_bytes += comm_round_bytes(ctx);
  launch_import(ctx);
  return 0;
}

// A round some shard produced more than xsz_cur runs for a peer in was held by k_import on
// every shard (each compares the same maxima). The send/recv of the rounds after it in the
// batch moved the same slots again and their kernels returned at once. Complete it: the
// whole slots, k_import again (which advances the window), and a larger exchange size.
int comm_complete_spill(sgn_ctx* ctx) {
  // some shard spilled runs past a slot: every shard grows its slots alike first
  if (ctx->h_ctrl->xhwm > ctx->S.xslot)
    if (int rc = grow_exchange_slot(ctx)) return rc;
  DevSim& S = ctx->S;
  hipStream_t st = ctx->stream;
  SGN_HIP(ctx, hipMemsetD32Async((hipDeviceptr_t)&S.ctrl->xsz, (int)S.xslot, 1, st));
  SGN_HIP(ctx, hipMemsetD32Async((hipDeviceptr_t)&S.ctrl->xspill, 0, 1, st));
  if (int rc = exchange(ctx, S.xslot)) return rc;
  ctx->x_bytes += (uint64_t)(ctx->nranks - 1) * ((uint64_t)(XHDR + S.xslot) * sizeof(EvRec));
  launch_import(ctx);
  uint64_t want = std::max<uint64_t>(2 * ctx->h_ctrl->xhwm, kXszInit);
  uint64_t sz = kXszInit;
  while (sz < want) sz <<= 1;
  ctx->xsz_cur = (uint32_t)std::min<uint64_t>(sz, S.xslot);
  SGN_HIP(ctx, hipMemsetD32Async((hipDeviceptr_t)&S.ctrl->xsz, (int)ctx->xsz_cur, 1, st));
  ctx->x_spills++;
  return ctrl_sync(ctx);
}

// Sharded APSP (routes.hip): every shard owns a contiguous block of rows (row tiles of the
// squaring matrix, or used sources of the final table) and the blocks are exchanged with one
// grouped in-place broadcast per step: shard r is the root of block r, so after the group
// every shard holds every block (an all-gather of blocks of unequal sizes).
int comm_bcast_blocks(sgn_ctx* ctx, void* base, size_t unit_bytes, const std::vector<uint64_t>& off) {
  ncclComm_t comm = (ncclComm_t)ctx->comm;
  ncclResult_t r = ncclGroupStart();
  for (uint32_t p = 0; p + 1 < off.size() && r == ncclSuccess; p++) {
    const size_t bytes = (size_t)(off[p + 1] - off[p]) * unit_bytes;
    if (!bytes) continue;
    char* b = (char*)base + (size_t)off[p] * unit_bytes;
    r = ncclBroadcast(b, b, bytes, ncclUint8, (int)p, comm, ctx->stream);
  }
  ncclResult_t r2 = ncclGroupEnd();
  if (r != ncclSuccess || r2 != ncclSuccess)
    return set_error(ctx, SGN_EDEVICE, std::string("RCCL row exchange: ") +
                                           ncclGetErrorString(r != ncclSuccess ? r : r2));
  return 0;
}

// In-place all-reduces of small device words: n_min u64 by min, then n_max u64 by max
// (one group).
int comm_allreduce_minmax(sgn_ctx* ctx, uint64_t* p, size_t n_min, size_t n_max) {
  ncclComm_t comm = (ncclComm_t)ctx->comm;
  ncclResult_t r = ncclGroupStart();
  if (n_min && r == ncclSuccess) r = ncclAllReduce(p, p, n_min, ncclUint64, ncclMin, comm, ctx->stream);
  if (n_max && r == ncclSuccess)
    r = ncclAllReduce(p + n_min, p + n_min, n_max, ncclUint64, ncclMax, comm, ctx->stream);
  ncclResult_t r2 = ncclGroupEnd();
  if (r != ncclSuccess || r2 != ncclSuccess)
    return set_error(ctx, SGN_EDEVICE, std::string("RCCL all-reduce: ") +
                                           ncclGetErrorString(r != ncclSuccess ? r : r2));
  return 0;
}

// ---- persistent multi-shard rounds, one shard per GPU: the peers' inboxes in this process ----
// Every shard exports its inbox (uncached device memory) as an IPC handle; one RCCL all-gather
// gives every shard every handle, and each opens its peers' (xGMI peer access). A shard that
// cannot export or open one tells the others through a max all-reduce, and then every shard
// keeps the per-round RCCL path (the same decision everywhere: the rounds stay in lockstep).
int comm_xpeer_map(sgn_ctx* ctx) {
  ncclComm_t comm = (ncclComm_t)ctx->comm;
  const uint32_t R = ctx->nranks;
  ctx->x_mapped = false;
  for (void* p : ctx->x_opened)
    if (p) (void)hipIpcCloseMemHandle(p);
  ctx->x_opened.clear();
  // per shard: its inbox handle and its GPU's PCI bus id (shards sharing one GPU — the one-GPU
  // RCCL rehearsal — would need their persistent grids resident side by side: only with
  // SGN_XPEER_SHARED=1, each grid sized for its share of the GPU; else the per-round path)
  static_assert(sizeof(hipIpcMemHandle_t) <= 64, "IPC handle size");
  constexpr size_t HB = 128;
  std::vector<uint8_t> mine(HB, 0), all((size_t)R * HB, 0);
  uint64_t bad = 0;
  hipIpcMemHandle_t h;
  if (!ctx->xin_mem || hipIpcGetMemHandle(&h, ctx->xin_mem) != hipSuccess)
    bad = 1;
  else
    std::memcpy(mine.data(), &h, sizeof(h));
  if (hipDeviceGetPCIBusId((char*)mine.data() + 64, 63, ctx->device) != hipSuccess) bad = 1;
  void* d = nullptr;
  SGN_HIP(ctx, hipMalloc(&d, (R + 1) * HB));
  hipError_t e = hipMemcpy(d, mine.data(), HB, hipMemcpyHostToDevice);
  ncclResult_t r = e == hipSuccess ? ncclAllGather(d, (char*)d + HB, HB, ncclUint8, comm, ctx->stream) : ncclInternalError;
  if (r == ncclSuccess) e = hipStreamSynchronize(ctx->stream);
  if (r == ncclSuccess && e == hipSuccess) e = hipMemcpy(all.data(), (char*)d + HB, (size_t)R * HB, hipMemcpyDeviceToHost);
  (void)hipFree(d);
  if (r != ncclSuccess) return set_error(ctx, SGN_EDEVICE, std::string("RCCL all-gather (inbox handles): ") + ncclGetErrorString(r));
  if (e != hipSuccess) return hip_fail(ctx, e, "inbox handle exchange");
  ctx->x_share = 0;
  for (uint32_t q = 0; q < R; q++)
    ctx->x_share += std::memcmp(all.data() + (size_t)q * HB + 64, mine.data() + 64, 64) == 0 ? 1u : 0u;
  const char* sh = getenv("SGN_XPEER_SHARED");
  if (ctx->x_share > 1 && !(sh && atoi(sh) == 1)) bad = 1;
  std::vector<char*> base(R, nullptr);
  base[ctx->rank] = (char*)ctx->xin_mem;
  for (uint32_t q = 0; q < R && !bad; q++) {
    if (q == ctx->rank) continue;
    hipIpcMemHandle_t hq;
    std::memcpy(&hq, all.data() + (size_t)q * HB, sizeof(hq));
    void* p = nullptr;
    if (hipIpcOpenMemHandle(&p, hq, hipIpcMemLazyEnablePeerAccess) != hipSuccess || !p) {
      bad = 1;
      (void)hipGetLastError();
      break;
    }
    ctx->x_opened.push_back(p);
    base[q] = (char*)p;
  }
  if (int rc = comm_allreduce_max_u64(ctx, &bad, 1)) return rc;
  if (bad) {  // some shard cannot map every inbox: all shards keep the per-round path
    for (void* p : ctx->x_opened)
      if (p) (void)hipIpcCloseMemHandle(p);
    ctx->x_opened.clear();
    ctx->x_off = true;
    return 0;
  }
  ctx->x_base = base;
  if (int rc = xpeer_upload(ctx)) return rc;
  ctx->x_mapped = true;
  return 0;
}

// Runs some shard sent past a peer's inbox slot (out[q]: this shard's for shard q) to their
// shards at a held round edge: the counts by one all-gather, the runs by one grouped send/recv.
int comm_xmove_spills(sgn_ctx* ctx, const std::vector<std::vector<EvRec>>& out, std::vector<EvRec>* in) {
  ncclComm_t comm = (ncclComm_t)ctx->comm;
  const uint32_t R = ctx->nranks, me = ctx->rank;
  std::vector<uint64_t> cnt(R, 0), all((size_t)R * R, 0);
  for (uint32_t q = 0; q < R; q++) cnt[q] = q < out.size() ? out[q].size() : 0;
  void* d = nullptr;
  SGN_HIP(ctx, hipMalloc(&d, (size_t)(R + R * R) * 8));
  SGN_HIP(ctx, hipMemcpy(d, cnt.data(), R * 8, hipMemcpyHostToDevice));
  ncclResult_t r = ncclAllGather(d, (uint64_t*)d + R, R, ncclUint64, comm, ctx->stream);
  if (r == ncclSuccess) SGN_HIP(ctx, hipStreamSynchronize(ctx->stream));
  if (r == ncclSuccess) SGN_HIP(ctx, hipMemcpy(all.data(), (uint64_t*)d + R, (size_t)R * R * 8, hipMemcpyDeviceToHost));
  (void)hipFree(d);
  if (r != ncclSuccess) return set_error(ctx, SGN_EDEVICE, std::string("RCCL all-gather (spill counts): ") + ncclGetErrorString(r));
  // all[q * R + p]: runs shard q holds for shard p
  uint64_t nout = 0, nin = 0;
  std::vector<uint64_t> ooff(R + 1, 0), ioff(R + 1, 0);
  for (uint32_t q = 0; q < R; q++) {
    ooff[q + 1] = ooff[q] + (q == me ? 0 : cnt[q]);
    ioff[q + 1] = ioff[q] + (q == me ? 0 : all[(size_t)q * R + me]);
  }
  nout = ooff[R];
  nin = ioff[R];
  in->assign(nin, EvRec{});
  if (nout == 0 && nin == 0) return 0;
  EvRec *ds = nullptr, *dr = nullptr;
  SGN_HIP(ctx, hipMalloc((void**)&ds, std::max<uint64_t>(1, nout) * sizeof(EvRec)));
  SGN_HIP(ctx, hipMalloc((void**)&dr, std::max<uint64_t>(1, nin) * sizeof(EvRec)));
  for (uint32_t q = 0; q < R; q++)
    if (q != me && cnt[q]) SGN_HIP(ctx, hipMemcpy(ds + ooff[q], out[q].data(), cnt[q] * sizeof(EvRec), hipMemcpyHostToDevice));
  r = ncclGroupStart();
  for (uint32_t q = 0; q < R && r == ncclSuccess; q++) {
    if (q == me) continue;
    if (ooff[q + 1] > ooff[q]) r = ncclSend(ds + ooff[q], (ooff[q + 1] - ooff[q]) * sizeof(EvRec), ncclUint8, (int)q, comm, ctx->stream);
    if (r == ncclSuccess && ioff[q + 1] > ioff[q])
      r = ncclRecv(dr + ioff[q], (ioff[q + 1] - ioff[q]) * sizeof(EvRec), ncclUint8, (int)q, comm, ctx->stream);
  }
  ncclResult_t r2 = ncclGroupEnd();
  hipError_t e = hipSuccess;
  if (r == ncclSuccess && r2 == ncclSuccess) e = hipStreamSynchronize(ctx->stream);
  if (r == ncclSuccess && r2 == ncclSuccess && e == hipSuccess && nin)
    e = hipMemcpy(in->data(), dr, nin * sizeof(EvRec), hipMemcpyDeviceToHost);
  (void)hipFree(ds);
  (void)hipFree(dr);
  if (r != ncclSuccess || r2 != ncclSuccess)
    return set_error(ctx, SGN_EDEVICE, std::string("RCCL send/recv (spilled runs): ") + ncclGetErrorString(r != ncclSuccess ? r : r2));
  if (e != hipSuccess) return hip_fail(ctx, e, "spilled runs exchange");
  return 0;
}

// max all-reduce of n host u64 values (through a device buffer)
int comm_allreduce_max_u64(sgn_ctx* ctx, uint64_t* host_v, size_t n) {
  void* d = nullptr;
  SGN_HIP(ctx, hipMalloc(&d, n * 8));
  hipError_t e = hipMemcpy(d, host_v, n * 8, hipMemcpyHostToDevice);
  ncclResult_t r = e == hipSuccess ? ncclAllReduce(d, d, n, ncclUint64, ncclMax, (ncclComm_t)ctx->comm, ctx->stream) : ncclInternalError;
  if (r == ncclSuccess) e = hipStreamSynchronize(ctx->stream);
  if (r == ncclSuccess && e == hipSuccess) e = hipMemcpy(host_v, d, n * 8, hipMemcpyDeviceToHost);
  (void)hipFree(d);
  if (r != ncclSuccess) return set_error(ctx, SGN_EDEVICE, std::string("RCCL all-reduce: ") + ncclGetErrorString(r));
  if (e != hipSuccess) return hip_fail(ctx, e, "all-reduce");
  return 0;
}

int comm_allreduce_max_u32(sgn_ctx* ctx, uint32_t* p, size_t n) {
  ncclResult_t r = ncclAllReduce(p, p, n, ncclUint32, ncclMax, (ncclComm_t)ctx->comm, ctx->stream);
  if (r != ncclSuccess) return set_error(ctx, SGN_EDEVICE, std::string("RCCL all-reduce: ") + ncclGetErrorString(r));
  return 0;
}

}  // namespace sgn

// ------------------------------------------------------------------------------------
// Local shard group: the same round-edge protocol between contexts of ONE process (any
// devices, e.g. several shards on one GPU), with device copies in place of RCCL. It runs
// the device-side multi-shard path (exchange slots, k_import, local finalize, window
// advance) exactly as the RCCL transport does, so it can be checked against a single
// shard on a one-GPU machine. Host-synchronous per round: a test transport, not a fast one.
// ------------------------------------------------------------------------------------
extern "C" {

int sgn_comm_init_local(sgn_ctx* const* ctxs, uint32_t n, uint64_t slot_events) {
  if (!ctxs || n < 2) return SGN_EINVAL;
  if (slot_events == 0 || slot_events > (1ULL << 26)) return SGN_EINVAL;
  for (uint32_t i = 0; i < n; i++) {
    sgn_ctx* c = ctxs[i];
    if (!c) return SGN_EINVAL;
    if (c->nranks != n || c->rank != i)
      return set_error(c, SGN_EINVAL, "local group: context i must be shard i of n");
    if (c->sim_ready) return set_error(c, SGN_ESTATE, "sgn_comm_init_local must precede sgn_sim_init");
  }
  for (uint32_t i = 0; i < n; i++) {
    ctxs[i]->comm_local = true;
    ctxs[i]->xslot = slot_events;
    ctxs[i]->group.assign(ctxs, ctxs + n);
  }
  return 0;
}

int sgn_run_local_group(sgn_ctx* const* ctxs, uint32_t n, uint64_t max_rounds, uint64_t* rounds_done) {
  if (!ctxs || n < 2) return SGN_EINVAL;
  for (uint32_t i = 0; i < n; i++)
    if (!ctxs[i] || !ctxs[i]->sim_ready || !ctxs[i]->comm_local || ctxs[i]->group.size() != n)
      return ctxs[i] ? set_error(ctxs[i], SGN_ESTATE, "not a local shard group") : SGN_EINVAL;
  for (uint32_t i = 0; i < n; i++)
    if (int rc = rng_release(ctxs[i])) return rc;
  // persistent rounds (k_rounds_x): every shard a range of workgroups of ONE launch on their GPU,
  // the inboxes ordinary (uncached) device memory of that GPU — the device code of the N-GPU
  // path, rehearsed on one GPU. SGN_LOCAL_PERSIST=0 keeps the per-round copies below.
  uint64_t pre = 0;
  {
    const char* lp = getenv("SGN_LOCAL_PERSIST");
    bool ok = !(lp && atoi(lp) == 0) && n <= XL_MAX;
    for (uint32_t i = 0; i < n && ok; i++)
      ok = ctxs[i]->device == ctxs[0]->device && xpersist_possible(ctxs[i]) && ctxs[i]->S.tkind == ctxs[0]->S.tkind;
    if (ok) {
      std::vector<sgn_ctx*> sh(ctxs, ctxs + n);
      if (!ctxs[0]->x_mapped) {
        std::vector<char*> base(n);
        for (uint32_t i = 0; i < n; i++) base[i] = (char*)ctxs[i]->xin_mem;
        for (uint32_t i = 0; i < n; i++) {
          ctxs[i]->x_base = base;
          if (int rc = xpeer_upload(ctxs[i])) return rc;
          ctxs[i]->x_mapped = true;
        }
      }
      if (int rc = run_xpersist(sh, false, max_rounds, &pre)) return rc;
      if (!ctxs[0]->x_off || pre >= max_rounds) {
        if (rounds_done) *rounds_done = pre;
        return 0;
      }
    }
  }
  max_rounds -= pre;
  // SGN_LOCAL_DEFER=1 (test hook): like the RCCL transport between its batch syncs, runs
  // k_import spilled stay in the spill area until a round is held (the next round's gathers
  // read them there)
  const char* dv = getenv("SGN_LOCAL_DEFER");
  const bool defer = dv && atoi(dv) == 1;
  uint64_t done = 0;
  for (; done < max_rounds; done++) {
    Ctrl h{};
    SGN_HIP(ctxs[0], hipMemcpy(&h, (const void*)ctxs[0]->S.ctrl, sizeof(Ctrl), hipMemcpyDeviceToHost));
    if (!h.active) break;
    for (uint32_t i = 0; i < n; i++) {
      SGN_HIP(ctxs[i], hipSetDevice(ctxs[i]->device));
      launch_execute(ctxs[i]);
    }
    for (uint32_t i = 0; i < n; i++) SGN_HIP(ctxs[i], hipStreamSynchronize(ctxs[i]->stream));
    // the all-to-all: shard b's receive slot and message a <- shard a's send slot and
    // message b (what comm_round_exchange's grouped send/recv does), then k_import everywhere
    auto exchange_import = [&]() -> int {
      for (uint32_t a = 0; a < n; a++) {
        sgn_ctx* A = ctxs[a];
        const size_t blk = (size_t)A->S.xslot + XHDR;
        for (uint32_t b = 0; b < n; b++) {
          if (b == a) continue;
          sgn_ctx* B = ctxs[b];
          uint64_t msg[4 * XHDR];
          SGN_HIP(A, hipMemcpy(msg, (const void*)(A->S.xout + (size_t)b * blk), sizeof(msg), hipMemcpyDeviceToHost));
          const uint64_t k = std::min<uint64_t>(msg[0], A->xslot);
          SGN_HIP(B, hipMemcpy((void*)(B->S.xin + (size_t)a * blk), (const void*)(A->S.xout + (size_t)b * blk),
                               (size_t)(XHDR + k) * sizeof(EvRec), hipMemcpyDefault));
        }
      }
      for (uint32_t i = 0; i < n; i++) {
        sgn_ctx* c = ctxs[i];
        SGN_HIP(c, hipSetDevice(c->device));
        launch_import(c);
        SGN_HIP(c, hipStreamSynchronize(c->stream));
      }
      return 0;
    };
    if (int rc = exchange_import()) return rc;
    // a round some shard spilled runs past a slot in was held by every shard alike: the slots
    // grow (the same size everywhere) and the round is exchanged and imported again
    if (int rc = ctrl_sync(ctxs[0])) return rc;
    if (ctxs[0]->h_ctrl->xspill) {
      for (uint32_t i = 0; i < n; i++) {
        sgn_ctx* c = ctxs[i];
        if (int rc = ctrl_sync(c)) return rc;
        if (c->h_ctrl->xhwm > c->S.xslot)
          if (int rc = grow_exchange_slot(c)) return rc;
        SGN_HIP(c, hipMemsetD32Async((hipDeviceptr_t)&c->S.ctrl->xspill, 0, 1, c->stream));
        SGN_HIP(c, hipMemsetD32Async((hipDeviceptr_t)&c->S.ctrl->xsz, (int)c->S.xslot, 1, c->stream));
        c->xsz_cur = c->S.xslot;
        SGN_HIP(c, hipStreamSynchronize(c->stream));
      }
      if (int rc = exchange_import()) return rc;
    }
    // a held round edge (the same on every shard) or a spill: the pools grow before the next
    bool held = false;
    for (uint32_t i = 0; i < n; i++) {
      if (int rc = ctrl_sync(ctxs[i])) return rc;
      held = held || ctxs[i]->h_ctrl->hold;
    }
    for (uint32_t i = 0; i < n && (held || !defer); i++)
      if (int rc = resolve_pools(ctxs[i])) return rc;
  }
  // (deferred spills: every run is back in its slab before the caller can ask for next-event
  // times — k_next_packet scans the pool and the extensions, not the spill area)
  if (defer)
    for (uint32_t i = 0; i < n; i++) {
      if (int rc = ctrl_sync(ctxs[i])) return rc;
      if (ctxs[i]->h_ctrl->spill_n || ctxs[i]->h_ctrl->hold)
        if (int rc = resolve_pools(ctxs[i])) return rc;
    }
  if (rounds_done) *rounds_done = pre + done;
  return 0;
}

}  // extern "C"

uint64_t sgn::layout_sig_comm() { return kLayoutSig; }
