// Column shards and row segments over RCCL for callers without a Python host
// (the Go shim).  Row segments: lx_rowseg_exchange at the end of this file,
// the driver of lx_rowseg_exchange.h over grouped ncclSend / ncclRecv.
//
// The multi-GPU protocol of DESIGN.md section 6, written against the public
// shard ABI (lx_shard_block / lx_shard_wire / lx_la_pack_dev / lx_la_unpack_dev /
// lx_la_own_dev / lx_forkless_cause_partial_dev / lx_fc_combine_dev), with the
// two collectives issued directly on the index handle's HIP stream:
//   * exchange: every (src -> dst) LowestAfter block in one ncclGroupStart /
//     ncclGroupEnd of ncclSend/ncclRecv (an all-to-all with uneven blocks),
//     each block at 1 byte per entry when it fits, else lx_shard_wire's width,
//     the widths announced first (one uint32 per peer);
//   * ForklessCause: partial stake sums -> ncclAllReduce(sum, uint32) ->
//     quorum test, stream-ordered (no host round trip).
// RCCL is resolved with dlopen/dlsym on first use so that loading the index
// library never pulls RCCL in, and a process that already holds RCCL (e.g.
// PyTorch's copy, same soname) reuses it.  The reference index is single-node
// (vecfc/index.go); this is the scale-out of the same computation.

#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <vector>

#include "lachesis_hip.h"
#include "lx_index.h"
#include "lx_rowseg_exchange.h"
#include "lx_shard_exchange.h"

namespace {

struct RcclApi {
    ncclResult_t (*GetUniqueId)(ncclUniqueId *) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    ncclResult_t (*Send)(const void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*AllReduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                              hipStream_t) = nullptr;
    ncclResult_t (*Broadcast)(const void *, void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    const char *(*ErrorString)(ncclResult_t) = nullptr;
    std::string error;
    bool ok = false;
};

RcclApi &rccl() {
    static RcclApi api;
    static std::once_flag once;
    std::call_once(once, [] {
        void *lib = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!lib) lib = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!lib) {
            api.error = std::string("cannot load RCCL: ") + dlerror();
            return;
        }
        bool all = true;
        auto get = [&](auto &fn, const char *name) {
            fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(lib, name));
            all &= fn != nullptr;
        };
        get(api.GetUniqueId, "ncclGetUniqueId");
        get(api.CommInitRank, "ncclCommInitRank");
        get(api.CommDestroy, "ncclCommDestroy");
        get(api.GroupStart, "ncclGroupStart");
        get(api.GroupEnd, "ncclGroupEnd");
        get(api.Send, "ncclSend");
        get(api.Recv, "ncclRecv");
        get(api.AllReduce, "ncclAllReduce");
        get(api.Broadcast, "ncclBroadcast");
        get(api.ErrorString, "ncclGetErrorString");
        api.ok = all;
        if (!all) api.error = "RCCL library lacks a required symbol";
    });
    return api;
}

thread_local std::string g_create_error;   // why the last lx_shard_comm_create failed (no handle to hold it)

int create_fail(int code, const std::string &msg) {
    g_create_error = msg;
    return code;
}

}  // namespace

struct lx_shard_comm {
    lx_index *ix = nullptr;
    ncclComm_t comm = nullptr;
    hipStream_t stream = nullptr;
    int device = 0;
    uint32_t rank = 0, nranks = 1;
    uint8_t *send = nullptr, *recv = nullptr;    // exchange staging (bytes), grown on demand
    size_t send_cap = 0, recv_cap = 0;
    uint8_t *mbuf = nullptr;                     // element-wise min of the dirty rows (incremental exchange)
    size_t mbuf_cap = 0;
    uint32_t *part = nullptr;                    // FC partial sums, grown on demand
    uint64_t part_cap = 0;
    uint8_t *ebuf = nullptr;                     // FC early exit: mask, idx, a, b, partials (grown on demand)
    size_t ecap = 0;
    uint64_t last_undecided = 0;                 // FC early exit: queries the last call sent to every shard
    uint32_t *wdev = nullptr;                    // wire widths: [0, G) sent, [G, 2G) received
    lx::ExchangeState xs;                        // byte-wire fallbacks remembered per destination
    bool rowseg = false;                         // a row-segment rank (lx_rowseg_comm_create)
    uint8_t *rbuf[lx::kRsBufs] = {};             // row-segment exchange buffers, grown on demand
    size_t rcap[lx::kRsBufs] = {};
    uint64_t *udev = nullptr;                    // row segments: [0, G) counts sent, [G, 2G) received, [2G] sum
    std::string err;

    int fail(int code, const char *fmt, ...) {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        err = buf;
        return code;
    }
    int hip(hipError_t e, const char *what) {
        if (e == hipSuccess) return 0;
        return fail(e == hipErrorOutOfMemory ? LX_ERR_NOMEM : LX_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
    }
    int nccl(ncclResult_t r, const char *what) {
        if (r == ncclSuccess) return 0;
        return fail(LX_ERR_HIP, "%s: %s", what, rccl().ErrorString(r));
    }
    int index(int rc, const char *what) {
        if (rc == 0) return 0;
        return fail(rc, "%s: %s", what, lx_last_error(ix));
    }
    int grow(uint8_t **p, size_t *cap, size_t need) {
        if (need <= *cap) return 0;
        if (*p) {
            (void)hipStreamSynchronize(stream);
            (void)hipFree(*p);
            *p = nullptr;
            *cap = 0;
        }
        if (int rc = hip(hipMalloc(reinterpret_cast<void **>(p), need), "hipMalloc")) return rc;
        *cap = need;
        return 0;
    }
};

#define LXC(call)                       \
    do {                                \
        if (int rc_ = (call)) return rc_; \
    } while (0)

extern "C" {

int lx_shard_comm_unique_id(uint8_t id[128]) {
    if (!id) return LX_ERR_ARG;
    RcclApi &api = rccl();
    if (!api.ok) return LX_ERR_HIP;
    ncclUniqueId u;
    if (api.GetUniqueId(&u) != ncclSuccess) return LX_ERR_HIP;
    static_assert(sizeof(u) == 128, "ncclUniqueId size");
    memcpy(id, &u, sizeof u);
    return 0;
}

static int comm_create(lx_index *h, const uint8_t id[128], uint32_t nranks, uint32_t rank, bool rowseg,
                       lx_shard_comm **out) {
    if (!h || !id || !out || rank >= nranks) return create_fail(LX_ERR_ARG, "bad argument");
    *out = nullptr;
    uint32_t srank = 0, scount = 1;
    if ((rowseg ? lx_rowseg_of(h, &srank, &scount) : lx_shard_of(h, &srank, &scount)))
        return create_fail(LX_ERR_ARG, "bad index handle");
    if (scount != nranks || srank != rank)
        return create_fail(LX_ERR_ARG, "rank " + std::to_string(rank) + " of " + std::to_string(nranks) +
                                           " does not match the handle's " + (rowseg ? "row segment " : "shard ") +
                                           std::to_string(srank) + " of " + std::to_string(scount));
    RcclApi &api = rccl();
    if (!api.ok) return create_fail(LX_ERR_HIP, api.error);
    auto *c = new lx_shard_comm();
    c->ix = h;
    c->rank = rank;
    c->nranks = nranks;
    c->rowseg = rowseg;
    void *stream = nullptr;
    std::string why;
    int rc = lx_device_planes(h, nullptr, nullptr, nullptr, &stream);
    c->stream = (hipStream_t)stream;
    hipDevice_t dev = 0;
    if (!rc && hipStreamGetDevice(c->stream, &dev) != hipSuccess) { rc = LX_ERR_HIP; why = "hipStreamGetDevice failed"; }
    c->device = dev;
    if (!rc && hipSetDevice(c->device) != hipSuccess) { rc = LX_ERR_HIP; why = "hipSetDevice failed"; }
    ncclUniqueId u;
    memcpy(&u, id, sizeof u);
    if (!rc) {
        const ncclResult_t r = api.CommInitRank(&c->comm, (int)nranks, u, (int)rank);
        if (r != ncclSuccess) {
            rc = LX_ERR_HIP;
            why = std::string("ncclCommInitRank: ") + api.ErrorString(r);
        }
    }
    if (rc) {
        delete c;
        return create_fail(rc, why);
    }
    *out = c;
    return 0;
}

int lx_shard_comm_create(lx_index *h, const uint8_t id[128], uint32_t nranks, uint32_t rank, lx_shard_comm **out) {
    return comm_create(h, id, nranks, rank, false, out);
}

int lx_rowseg_comm_create(lx_index *h, const uint8_t id[128], uint32_t nranks, uint32_t rank, lx_shard_comm **out) {
    return comm_create(h, id, nranks, rank, true, out);
}

void lx_shard_comm_destroy(lx_shard_comm *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->comm) rccl().CommDestroy(c->comm);
    (void)hipFree(c->send);
    (void)hipFree(c->recv);
    (void)hipFree(c->mbuf);
    (void)hipFree(c->part);
    (void)hipFree(c->ebuf);
    (void)hipFree(c->wdev);
    for (uint8_t *p : c->rbuf) (void)hipFree(p);
    (void)hipFree(c->udev);
    delete c;
}

int lx_shard_fc_undecided(const lx_shard_comm *c, uint64_t *undecided) {
    if (!c || !undecided) return LX_ERR_ARG;
    *undecided = c->last_undecided;
    return 0;
}

const char *lx_shard_comm_last_error(const lx_shard_comm *c) {
    return c ? c->err.c_str() : g_create_error.c_str();   // NULL: why the last create failed
}

// the index side of the exchange driver (lx_shard_exchange.h) over the shard ABI
struct RcclOps {
    lx_shard_comm *c;
    int block(uint32_t s, uint32_t d, uint64_t *n) { return c->index(lx_shard_block(c->ix, s, d, n), "lx_shard_block"); }
    int wire(uint32_t *w) { return c->index(lx_shard_wire(c->ix, w), "lx_shard_wire"); }
    int pack(uint32_t d, uint8_t *buf, uint32_t w) {
        const int rc = lx_la_pack_wire_dev(c->ix, d, buf, w);
        return rc == LX_ERR_WIRE ? rc : c->index(rc, "lx_la_pack_wire_dev");
    }
    int unpack(uint32_t s, const uint8_t *buf, uint32_t w) {
        return c->index(lx_la_unpack_wire_dev(c->ix, s, buf, w), "lx_la_unpack_wire_dev");
    }
    int own() { return c->index(lx_la_own_dev(c->ix, nullptr), "lx_la_own_dev"); }
    int branches(uint32_t *nb) {
        *nb = lx_num_branches(c->ix);
        return 0;
    }
    int dirty(uint32_t nb, uint32_t *dmin) { return c->index(lx_shard_dirty(c->ix, nb, dmin), "lx_shard_dirty"); }
    int dirty_set(uint32_t nb, const uint32_t *dmin) {
        return c->index(lx_shard_dirty_set(c->ix, nb, dmin), "lx_shard_dirty_set");
    }
    int commit() { return c->index(lx_shard_dirty_commit(c->ix), "lx_shard_dirty_commit"); }
    uint8_t *send_buf(size_t n) { return c->grow(&c->send, &c->send_cap, std::max<size_t>(n, 1)) ? nullptr : c->send; }
    uint8_t *recv_buf(size_t n) { return c->grow(&c->recv, &c->recv_cap, std::max<size_t>(n, 1)) ? nullptr : c->recv; }
};

// the collectives: grouped ncclSend / ncclRecv on the index stream; ncclGroupEnd
// is called on every path once ncclGroupStart succeeded (an error inside the
// group must not leave the thread in RCCL group mode)
struct RcclNet {
    lx_shard_comm *c;
    int group(const std::function<int()> &body) {
        RcclApi &api = rccl();
        int rc = c->nccl(api.GroupStart(), "ncclGroupStart");
        if (rc) return rc;
        rc = body();
        const int rc2 = c->nccl(api.GroupEnd(), "ncclGroupEnd");
        return rc ? rc : rc2;
    }
    int widths(const uint32_t *sw, uint32_t *rw) {
        RcclApi &api = rccl();
        const uint32_t G = c->nranks, r = c->rank;
        LXC(c->hip(hipMemcpyAsync(c->wdev, sw, 4ull * G, hipMemcpyHostToDevice, c->stream), "hipMemcpyAsync"));
        LXC(group([&] {
            for (uint32_t q = 0; q < G; q++) {
                if (q == r) continue;
                LXC(c->nccl(api.Send(c->wdev + q, 1, ncclUint32, (int)q, c->comm, c->stream), "ncclSend"));
                LXC(c->nccl(api.Recv(c->wdev + G + q, 1, ncclUint32, (int)q, c->comm, c->stream), "ncclRecv"));
            }
            return 0;
        }));
        LXC(c->hip(hipMemcpyAsync(rw, c->wdev + G, 4ull * G, hipMemcpyDeviceToHost, c->stream), "hipMemcpyAsync"));
        return c->hip(hipStreamSynchronize(c->stream), "hipStreamSynchronize");
    }
    int min_u32(uint32_t *v, uint32_t n) {
        LXC(c->grow(&c->mbuf, &c->mbuf_cap, 4ull * n));
        LXC(c->hip(hipMemcpyAsync(c->mbuf, v, 4ull * n, hipMemcpyHostToDevice, c->stream), "hipMemcpyAsync"));
        LXC(c->nccl(rccl().AllReduce(c->mbuf, c->mbuf, n, ncclUint32, ncclMin, c->comm, c->stream), "ncclAllReduce"));
        LXC(c->hip(hipMemcpyAsync(v, c->mbuf, 4ull * n, hipMemcpyDeviceToHost, c->stream), "hipMemcpyAsync"));
        return c->hip(hipStreamSynchronize(c->stream), "hipStreamSynchronize");
    }
    int blocks(const uint8_t *send, const uint64_t *so, const uint64_t *sb, uint8_t *recv, const uint64_t *ro,
               const uint64_t *rb) {
        RcclApi &api = rccl();
        const uint32_t G = c->nranks, r = c->rank;
        return group([&] {
            for (uint32_t q = 0; q < G; q++) {
                if (q == r) continue;
                // blocks may be empty (a shard without rows yet): zero-byte send/recv keep the pairing
                LXC(c->nccl(api.Send(send + so[q], sb[q], ncclUint8, (int)q, c->comm, c->stream), "ncclSend"));
                LXC(c->nccl(api.Recv(recv + ro[q], rb[q], ncclUint8, (int)q, c->comm, c->stream), "ncclRecv"));
            }
            return 0;
        });
    }
};

int lx_shard_exchange(lx_shard_comm *c) {
    if (!c) return LX_ERR_ARG;
    if (c->rowseg) return c->fail(LX_ERR_STATE, "a row-segment communicator (lx_rowseg_exchange)");
    LXC(c->hip(hipSetDevice(c->device), "hipSetDevice"));
    const uint32_t G = c->nranks;
    if (G == 1) return 0;   // an unsharded handle holds whole LowestAfter rows already
    if (!c->wdev) LXC(c->hip(hipMalloc(reinterpret_cast<void **>(&c->wdev), 8ull * G), "hipMalloc"));
    RcclOps ops{c};
    RcclNet net{c};
    c->err.clear();
    const int rc = lx::shard_exchange_run(ops, net, c->rank, G, c->xs);
    if (rc) {
        if (c->err.empty()) c->fail(rc, "exchange failed (%d): block sizes or wire widths disagree between ranks", rc);
        return rc;
    }
    // the unpacks ran on the handle's stream after the received bytes landed
    return c->hip(hipStreamSynchronize(c->stream), "hipStreamSynchronize");
}

// Block layout shared by every implementation of the exchange (lx_shard_exchange.h).
int lx_shard_exchange_layout(uint32_t G, uint32_t self, const uint64_t *entries, const uint32_t *width,
                             uint64_t *off) {
    if (!G || self >= G || !entries || !width || !off) return LX_ERR_ARG;
    lx::shard_layout(G, self, entries, width, off);
    return 0;
}

// the early exit's fixed cost (a broadcast, a scan, a host round trip) pays
// from this many queries on (smaller calls: the FC cache's fills, one pair)
constexpr uint64_t kShardEarlyMin = 1ull << 14;

int lx_forkless_cause_sharded_dev(lx_shard_comm *c, uint64_t n, const uint32_t *a, const uint32_t *b, uint8_t *out) {
    if (!c || (n && (!a || !b || !out))) return LX_ERR_ARG;
    if (c->rowseg) return c->fail(LX_ERR_STATE, "row segments answer ForklessCause through the index");
    if (!n) return 0;
    RcclApi &api = rccl();
    LXC(c->hip(hipSetDevice(c->device), "hipSetDevice"));
    if (c->nranks == 1)
        return c->index(lx_forkless_cause_batch_dev(c->ix, n, a, b, out, nullptr), "lx_forkless_cause_batch_dev");
    if (n > c->part_cap) {
        uint8_t *p = reinterpret_cast<uint8_t *>(c->part);
        size_t cap = c->part_cap * 4;
        LXC(c->grow(&p, &cap, n * 4));
        c->part = reinterpret_cast<uint32_t *>(p);
        c->part_cap = n;
    }
    if (n >= kShardEarlyMin && lx_fc_shard_early(c->ix, nullptr)) {
        // early exit: shard 0 decides most queries alone, the
        // others add partials for the rest only
        const uint64_t W = (n + 63) / 64;
        LXC(c->grow(&c->ebuf, &c->ecap, 16 * W + 16 * n));
        uint64_t *mask = reinterpret_cast<uint64_t *>(c->ebuf);
        uint32_t *idx = reinterpret_cast<uint32_t *>(c->ebuf + 16 * W);
        uint32_t *a2 = idx + n, *b2 = a2 + n, *p2 = b2 + n;
        const bool s0 = c->rank == 0;
        if (s0) {
            LXC(c->index(lx_forkless_cause_partial_dev(c->ix, n, a, b, c->part, nullptr), "lx_forkless_cause_partial_dev"));
            LXC(c->index(lx_fc_shard_decide_dev(c->ix, n, c->part, mask, nullptr), "lx_fc_shard_decide_dev"));
        }
        LXC(c->nccl(api.Broadcast(mask, mask, 2 * W, ncclUint64, 0, c->comm, c->stream), "ncclBroadcast"));
        LXC(c->hip(hipStreamSynchronize(c->stream), "hipStreamSynchronize"));
        uint64_t m = 0;
        LXC(c->index(lx_fc_shard_undecided_dev(c->ix, n, mask, a, b, s0 ? c->part : nullptr, idx, a2, b2,
                                               s0 ? p2 : nullptr, &m), "lx_fc_shard_undecided_dev"));
        c->last_undecided = m;
        if (m) {
            if (!s0) LXC(c->index(lx_forkless_cause_partial_dev(c->ix, m, a2, b2, p2, nullptr), "lx_forkless_cause_partial_dev"));
            LXC(c->nccl(api.AllReduce(p2, p2, m, ncclUint32, ncclSum, c->comm, c->stream), "ncclAllReduce"));
        }
        LXC(c->index(lx_fc_shard_answer_dev(c->ix, n, mask, m, idx, p2, out, nullptr), "lx_fc_shard_answer_dev"));
        return 0;
    }
    c->last_undecided = n;
    LXC(c->index(lx_forkless_cause_partial_dev(c->ix, n, a, b, c->part, nullptr), "lx_forkless_cause_partial_dev"));
    LXC(c->nccl(api.AllReduce(c->part, c->part, n, ncclUint32, ncclSum, c->comm, c->stream), "ncclAllReduce"));
    LXC(c->index(lx_fc_combine_dev(c->ix, n, c->part, out, nullptr), "lx_fc_combine_dev"));
    return 0;
}

int lx_shard_get_rows(lx_shard_comm *c, uint32_t mode, uint64_t n, const uint32_t *ev, uint8_t *out, uint64_t slot,
                      uint32_t *len) {
    if (!c || mode > 2 || (n && (!ev || !out || !len))) return LX_ERR_ARG;
    if (c->rowseg) return c->fail(LX_ERR_STATE, "row segments route their getters (lx_rowseg_get_rows)");
    if (n > 0xFFFFFFFFull) return c->fail(LX_ERR_ARG, "too many rows in one call");
    if (n && (slot < 8ull * std::max(c->ix->B, c->ix->V) || slot % 16))
        return c->fail(LX_ERR_ARG, "row slot of %llu bytes: needs >= %llu and a multiple of 16",
                       (unsigned long long)slot, 8ull * std::max(c->ix->B, c->ix->V));
    if (!n) return 0;
    RcclApi &api = rccl();
    LXC(c->hip(hipSetDevice(c->device), "hipSetDevice"));
    // this shard's branches, zeros elsewhere (completed on return) ...
    LXC(c->index(lx_get_rows_dev(c->ix, mode, (uint32_t)n, ev, out, slot, len), "lx_get_rows_dev"));
    if (c->nranks == 1) return 0;
    // ... summed word by word over the shards (each word has one writer), and
    // the longest length any shard's entries imply
    LXC(c->nccl(api.AllReduce(out, out, n * slot / 4, ncclUint32, ncclSum, c->comm, c->stream), "ncclAllReduce"));
    LXC(c->nccl(api.AllReduce(len, len, n, ncclUint32, ncclMax, c->comm, c->stream), "ncclAllReduce"));
    return c->hip(hipStreamSynchronize(c->stream), "hipStreamSynchronize");
}

// ---- row segments: the driver of lx_rowseg_exchange.h over the rowseg ABI
struct RcclRowOps {
    lx_shard_comm *c;
    int row_words(uint32_t *w) { return c->index(lx_rowseg_row_words(c->ix, w), "lx_rowseg_row_words"); }
    int request_cap(uint32_t *cap) { return c->index(lx_rowseg_request_cap(c->ix, cap), "lx_rowseg_request_cap"); }
    int requests(uint32_t *ids, uint32_t cap, uint32_t *counts) {
        return c->index(lx_rowseg_requests(c->ix, ids, cap, counts), "lx_rowseg_requests");
    }
    int serve(uint32_t n, const uint32_t *ids, uint32_t *rows, uint32_t *ready) {
        return c->index(lx_rowseg_serve(c->ix, n, ids, rows, ready), "lx_rowseg_serve");
    }
    int receive(uint32_t n, const uint32_t *ids, const uint32_t *rows, const uint32_t *ready) {
        return c->index(lx_rowseg_receive(c->ix, n, ids, rows, ready, nullptr), "lx_rowseg_receive");
    }
    int la(uint64_t *counts) { return c->index(lx_rowseg_la(c->ix, counts), "lx_rowseg_la"); }
    int la_fetch(uint32_t *buf) { return c->index(lx_rowseg_la_fetch(c->ix, buf), "lx_rowseg_la_fetch"); }
    int la_apply(uint64_t n, const uint32_t *buf) { return c->index(lx_rowseg_la_apply(c->ix, n, buf), "lx_rowseg_la_apply"); }
    int finish() { return c->index(lx_rowseg_finish(c->ix), "lx_rowseg_finish"); }
    void *buf(int k, size_t bytes) { return c->grow(&c->rbuf[k], &c->rcap[k], bytes) ? nullptr : c->rbuf[k]; }
    // ForklessCause across ranks (rowseg_fc_run)
    uint32_t rank() const { return c->rank; }
    int fc_route(uint64_t n, const uint32_t *qa, const uint32_t *qb, uint32_t *ra, uint32_t *rb, uint32_t *perm,
                 uint64_t *counts) {
        return c->index(lx_rowseg_fc_route(c->ix, n, qa, qb, ra, rb, perm, counts), "lx_rowseg_fc_route");
    }
    int fc_need(uint64_t m, const uint32_t *ra, const uint32_t *rb, uint32_t *ids, uint64_t cap, uint64_t *counts) {
        return c->index(lx_rowseg_fc_need(c->ix, m, ra, rb, ids, cap, counts), "lx_rowseg_fc_need");
    }
    int la_serve(uint64_t n, const uint32_t *ids, uint32_t *rows) {
        return c->index(lx_rowseg_la_serve(c->ix, n, ids, rows), "lx_rowseg_la_serve");
    }
    int la_store(uint64_t n, const uint32_t *ids, const uint32_t *rows) {
        return c->index(lx_rowseg_la_store(c->ix, n, ids, rows), "lx_rowseg_la_store");
    }
    int fc_pairs(uint64_t m, const uint32_t *a, const uint32_t *b, uint8_t *ans) {
        LXC(c->index(lx_forkless_cause_batch_dev(c->ix, m, a, b, ans, nullptr), "lx_forkless_cause_batch_dev"));
        return c->index(lx_sync(c->ix), "lx_sync");
    }
    int fc_unroute(uint64_t n, const uint32_t *perm, const uint8_t *ans, uint8_t *out) {
        return c->index(lx_rowseg_fc_unroute(c->ix, n, perm, ans, out), "lx_rowseg_fc_unroute");
    }
    int get_rows(uint32_t mode, uint64_t m, const uint32_t *ids, uint8_t *rows, uint64_t slot, uint32_t *lens) {
        if (m > 0xFFFFFFFFull) return c->fail(LX_ERR_ARG, "too many rows in one call");
        return c->index(lx_get_rows_dev(c->ix, mode, (uint32_t)m, ids, rows, slot, lens), "lx_get_rows_dev");
    }
    int rows_unroute(uint64_t n, const uint32_t *perm, const uint8_t *rows, uint64_t slot, const uint32_t *lens,
                     uint8_t *out, uint32_t *out_len) {
        return c->index(lx_rowseg_rows_unroute(c->ix, n, perm, rows, slot, lens, out, out_len),
                        "lx_rowseg_rows_unroute");
    }
};

// the collectives on the handle's stream; the own block moves by a local copy
struct RcclRowNet {
    lx_shard_comm *c;
    RcclNet group_net{c};
    int sum(uint64_t x, uint64_t *all) {
        const uint32_t G = c->nranks;
        LXC(c->hip(hipMemcpyAsync(c->udev + 2 * G, &x, 8, hipMemcpyHostToDevice, c->stream), "hipMemcpyAsync"));
        LXC(c->nccl(rccl().AllReduce(c->udev + 2 * G, c->udev + 2 * G, 1, ncclUint64, ncclSum, c->comm, c->stream),
                    "ncclAllReduce"));
        LXC(c->hip(hipMemcpyAsync(all, c->udev + 2 * G, 8, hipMemcpyDeviceToHost, c->stream), "hipMemcpyAsync"));
        return c->hip(hipStreamSynchronize(c->stream), "hipStreamSynchronize");
    }
    int counts(const uint64_t *send, uint64_t *recv) {
        RcclApi &api = rccl();
        const uint32_t G = c->nranks, r = c->rank;
        LXC(c->hip(hipMemcpyAsync(c->udev, send, 8ull * G, hipMemcpyHostToDevice, c->stream), "hipMemcpyAsync"));
        LXC(group_net.group([&] {
            for (uint32_t q = 0; q < G; q++) {
                if (q == r) continue;
                LXC(c->nccl(api.Send(c->udev + q, 1, ncclUint64, (int)q, c->comm, c->stream), "ncclSend"));
                LXC(c->nccl(api.Recv(c->udev + G + q, 1, ncclUint64, (int)q, c->comm, c->stream), "ncclRecv"));
            }
            return 0;
        }));
        LXC(c->hip(hipMemcpyAsync(recv, c->udev + G, 8ull * G, hipMemcpyDeviceToHost, c->stream), "hipMemcpyAsync"));
        LXC(c->hip(hipStreamSynchronize(c->stream), "hipStreamSynchronize"));
        recv[r] = send[r];
        return 0;
    }
    int move(const void *send, const uint64_t *sb, void *recv, const uint64_t *rb) {
        RcclApi &api = rccl();
        const uint32_t G = c->nranks, r = c->rank;
        std::vector<uint64_t> so(G + 1, 0), ro(G + 1, 0);
        for (uint32_t q = 0; q < G; q++) so[q + 1] = so[q] + sb[q], ro[q + 1] = ro[q] + rb[q];
        const uint8_t *s = static_cast<const uint8_t *>(send);
        uint8_t *d = static_cast<uint8_t *>(recv);
        if (sb[r] != rb[r]) return c->fail(LX_ERR_STATE, "row-segment exchange: own block %llu != %llu bytes",
                                          (unsigned long long)sb[r], (unsigned long long)rb[r]);
        if (sb[r])
            LXC(c->hip(hipMemcpyAsync(d + ro[r], s + so[r], sb[r], hipMemcpyDeviceToDevice, c->stream),
                       "hipMemcpyAsync"));
        return group_net.group([&] {
            for (uint32_t q = 0; q < G; q++) {
                if (q == r) continue;
                LXC(c->nccl(api.Send(s + so[q], sb[q], ncclUint8, (int)q, c->comm, c->stream), "ncclSend"));
                LXC(c->nccl(api.Recv(d + ro[q], rb[q], ncclUint8, (int)q, c->comm, c->stream), "ncclRecv"));
            }
            return 0;
        });
    }
};

// A whole index (no row segments) on a one-rank communicator: nothing to
// join, the calls go straight to the index.  A row-segment handle (seg_count
// >= 1) before its batch is not whole: LX_ERR_STATE, as every step out of order.
static int rs_whole(lx_shard_comm *c, bool *whole) {
    *whole = c->nranks == 1 && !c->ix->rowseg();
    if (c->ix->rowseg() && !c->ix->rs_state)
        return c->fail(LX_ERR_STATE, "row-segment handle has no batch yet (lx_add_batch first)");
    return 0;
}

int lx_rowseg_exchange(lx_shard_comm *c, uint64_t stats[4]) {
    if (!c) return LX_ERR_ARG;
    if (!c->rowseg) return c->fail(LX_ERR_STATE, "not a row-segment communicator (lx_rowseg_comm_create)");
    LXC(c->hip(hipSetDevice(c->device), "hipSetDevice"));
    const uint32_t G = c->nranks;
    bool whole = false;
    LXC(rs_whole(c, &whole));
    if (whole) return 0;   // a whole index: nothing to join
    if (!c->udev) LXC(c->hip(hipMalloc(reinterpret_cast<void **>(&c->udev), 8ull * (2 * G + 1)), "hipMalloc"));
    RcclRowOps ops{c};
    RcclRowNet net{c};
    c->err.clear();
    lx::RowsegExchangeStats st;
    const int rc = lx::rowseg_exchange_run(ops, net, G, st);
    if (rc) {
        if (c->err.empty()) c->fail(rc, "row-segment exchange failed (%d)", rc);
        return rc;
    }
    if (stats) {
        stats[0] = st.rounds;
        stats[1] = st.rows_received;
        stats[2] = st.la_sent;
        stats[3] = st.la_received;
    }
    return 0;
}

int lx_rowseg_forkless_cause(lx_shard_comm *c, uint64_t n, const uint32_t *qa, const uint32_t *qb, uint8_t *out,
                             uint64_t stats[4]) {
    if (!c) return LX_ERR_ARG;
    if (!c->rowseg) return c->fail(LX_ERR_STATE, "not a row-segment communicator (lx_rowseg_comm_create)");
    LXC(c->hip(hipSetDevice(c->device), "hipSetDevice"));
    const uint32_t G = c->nranks;
    bool whole = false;
    LXC(rs_whole(c, &whole));
    if (whole) {
        LXC(c->index(lx_forkless_cause_batch_dev(c->ix, n, qa, qb, out, nullptr), "lx_forkless_cause_batch_dev"));
        return c->index(lx_sync(c->ix), "lx_sync");
    }
    if (!c->udev) LXC(c->hip(hipMalloc(reinterpret_cast<void **>(&c->udev), 8ull * (2 * G + 1)), "hipMalloc"));
    RcclRowOps ops{c};
    RcclRowNet net{c};
    c->err.clear();
    lx::RowsegFcStats st;
    const int rc = lx::rowseg_fc_run(ops, net, G, n, qa, qb, out, st);
    if (rc) {
        if (c->err.empty()) c->fail(rc, "row-segment ForklessCause failed (%d)", rc);
        return rc;
    }
    if (stats) {
        stats[0] = st.routed_away;
        stats[1] = st.answered;
        stats[2] = st.rows_received;
        stats[3] = st.rows_sent;
    }
    return 0;
}

int lx_rowseg_get_rows(lx_shard_comm *c, uint32_t mode, uint64_t n, const uint32_t *ev, uint8_t *out, uint64_t slot,
                       uint32_t *len) {
    if (!c || mode > 2 || (n && (!ev || !out || !len))) return LX_ERR_ARG;
    if (!c->rowseg) return c->fail(LX_ERR_STATE, "not a row-segment communicator (lx_rowseg_comm_create)");
    LXC(c->hip(hipSetDevice(c->device), "hipSetDevice"));
    const uint32_t G = c->nranks;
    // one slot rule for both paths, checked before any collective: a slot
    // holds the longest row (8 B per branch, HB) and is a multiple of 16 B
    // (lx_rowseg_rows_unroute)
    if (n && (slot < 8ull * std::max(c->ix->B, c->ix->V) || slot % 16))
        return c->fail(LX_ERR_ARG, "row slot of %llu bytes: needs >= %llu and a multiple of 16",
                       (unsigned long long)slot, 8ull * std::max(c->ix->B, c->ix->V));
    bool whole = false;
    LXC(rs_whole(c, &whole));
    if (whole) {
        if (n > 0xFFFFFFFFull) return c->fail(LX_ERR_ARG, "too many rows in one call");
        return c->index(lx_get_rows_dev(c->ix, mode, (uint32_t)n, ev, out, slot, len), "lx_get_rows_dev");
    }
    if (!c->udev) LXC(c->hip(hipMalloc(reinterpret_cast<void **>(&c->udev), 8ull * (2 * G + 1)), "hipMalloc"));
    RcclRowOps ops{c};
    RcclRowNet net{c};
    c->err.clear();
    const int rc = lx::rowseg_get_run(ops, net, G, mode, n, ev, out, slot, len);
    if (rc && c->err.empty()) c->fail(rc, "row-segment getters failed (%d)", rc);
    return rc;
}

}  // extern "C"
