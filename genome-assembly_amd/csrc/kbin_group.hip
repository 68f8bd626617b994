// kbin_group.hip -- multi-GPU groups behind the C-ABI (include/kbin.h,
// "multi-GPU groups").
//
// The canonical-mmer space shards: every (mmer, kmer) entry of binning.c's
// two-level table (level 1 keyed by the signature mmer, binning.c:1045;
// prune_kmers per mmer table, binning.c:1085) lives on rank owner(mmer), so
// the ranks' results are disjoint and their union is the single-GPU result.
// A group is G ranks; each holds
//   sender   : a kb_ctx with this rank's reads; kb_route_scatter writes its
//              super-k-mer records into one region per destination rank
//   exchange : the per-destination counts (all-gather), then the records
//              (grouped point-to-point send/recv), over RCCL (xGMI); or, when
//              every rank lives in this process on one device (virtual shards
//              for tests on one GPU), device copies on the same code path
//   receiver : a kb_ctx that adopts the records it got, concatenated by source
//              rank (kb_submit_superkmers_device), and bins them (kb_finalize)
// Two region / receive slots let the exchange of one unit overlap the
// binning of the previous one (kb_group_send / kb_group_receive).
//
// Ranks either all live in one process (kb_group_create: one host thread
// drives every device; RCCL communicators from ncclCommInitAll) or one per
// process (kb_group_create_rank: ncclCommInitRank with a unique id the caller
// distributes).  RCCL is loaded at run time (dlopen of librccl.so.1): a
// process that never forms an RCCL group does not load it, and one that has
// it loaded already (torch) shares that copy.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <algorithm>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/kbin.h"
#include "kbin_internal.h"

namespace {

thread_local std::string g_gerr;  // (also handed to kb_last_error)

// ---- RCCL entry points, resolved once
struct Rccl {
    bool ok = false;
    std::string why;
    decltype(&ncclGetUniqueId) GetUniqueId = nullptr;
    decltype(&ncclCommInitRank) CommInitRank = nullptr;
    decltype(&ncclCommInitAll) CommInitAll = nullptr;
    decltype(&ncclCommDestroy) CommDestroy = nullptr;
    decltype(&ncclGetErrorString) GetErrorString = nullptr;
    decltype(&ncclAllGather) AllGather = nullptr;
    decltype(&ncclSend) Send = nullptr;
    decltype(&ncclRecv) Recv = nullptr;
    decltype(&ncclGroupStart) GroupStart = nullptr;
    decltype(&ncclGroupEnd) GroupEnd = nullptr;
};

Rccl& rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        const char* names[] = {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
        void* h = nullptr;
        for (const char* n : names)
            if ((h = dlopen(n, RTLD_NOW | RTLD_GLOBAL))) break;
        if (!h) {
            r.why = std::string("dlopen librccl.so.1: ") + dlerror();
            return;
        }
#define KB_SYM(f)                                                              \
    r.f = reinterpret_cast<decltype(r.f)>(dlsym(h, "nccl" #f));                \
    if (!r.f) {                                                                \
        r.why = "librccl: no symbol nccl" #f;                                  \
        return;                                                                \
    }
        KB_SYM(GetUniqueId) KB_SYM(CommInitRank) KB_SYM(CommInitAll) KB_SYM(CommDestroy) KB_SYM(GetErrorString)
        KB_SYM(AllGather) KB_SYM(Send) KB_SYM(Recv) KB_SYM(GroupStart) KB_SYM(GroupEnd)
#undef KB_SYM
        r.ok = true;
    });
    return r;
}

int gfail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_gerr = buf;
    kb::set_last_error(buf);
    return code;
}

#define GHIP(expr)                                                                                  \
    do {                                                                                            \
        hipError_t _e = (expr);                                                                     \
        if (_e != hipSuccess)                                                                       \
            return gfail(_e == hipErrorOutOfMemory ? KB_ENOMEM : KB_EDEVICE, "%s: %s (%s:%d)", #expr, \
                         hipGetErrorString(_e), __FILE__, __LINE__);                                \
    } while (0)
#define GNCCL(expr)                                                                                      \
    do {                                                                                                 \
        ncclResult_t _r = (expr);                                                                        \
        if (_r != ncclSuccess)                                                                           \
            return gfail(KB_EDEVICE, "%s: %s (%s:%d)", #expr, rccl().GetErrorString(_r), __FILE__, __LINE__); \
    } while (0)
#define GKB(expr)                                                                   \
    do {                                                                            \
        int _rc = (expr);                                                           \
        if (_rc != KB_OK) return gfail(_rc, "%s: %s", #expr, kb_last_error());     \
    } while (0)

struct GBuf {  // device words, grown on demand (1/8 headroom)
    uint64_t* p = nullptr;
    uint64_t cap = 0;
    int dev = 0;
    hipError_t ensure(uint64_t n) {
        if (n <= cap && p) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        const uint64_t want = std::max<uint64_t>(n, 1) + n / 8;
        hipError_t e = hipMalloc((void**)&p, want * sizeof(uint64_t));
        if (e == hipSuccess) cap = want;
        else p = nullptr;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

constexpr int SLOTS = 2;

struct Unit {  // one send in flight (a slot)
    bool busy = false;
    uint32_t part = 0, n_parts = 1;
    std::vector<uint64_t> C;  // [G * G] counts: C[s * G + d] records from rank s to rank d
    // the send stage (route, counts, records) runs on the group's sender
    // thread: done once it has returned, rc / err its outcome
    bool done = true;
    int rc = KB_OK;
    std::string err;
};

struct Rank {
    int dev = 0;
    int grank = 0;  // global rank
    kb_ctx* send = nullptr;
    kb_ctx* recv = nullptr;
    ncclComm_t comm = nullptr;
    hipStream_t xs = nullptr;  // exchange stream
    hipEvent_t landed[SLOTS] = {};  // the slot's records received (and its sends done)
    hipEvent_t routed = nullptr;    // the sender stream's routing of the unit being sent
    GBuf regions[SLOTS], rbuf[SLOTS];
    GBuf cdev;                  // [G + 1] this rank's row, then [G * (G + 1)] every rank's (all-gather)
    uint64_t* h_counts = nullptr;  // pinned [G * (G + 1)]: row s = rank s's G counts + its routing status
    int route_rc = KB_OK;       // this unit's routing outcome (travels with the counts)
    uint64_t cap = 0;           // region capacity (records per destination), learned
    bool ordered = false;       // plan/pack sender (destination-major, read order)
    std::vector<uint64_t> soff[SLOTS];  // the slot's first record per destination
    uint64_t n_reads = 0;       // reads submitted since the last kb_group_reset
    std::string err;            // a worker thread's failure
};

}  // namespace

struct kb_group {
    kb_params p{};
    int G = 1;            // ranks in the group
    bool local = false;   // device-copy transport (every rank in this process)
    // host transport (kb_group_create_rank_host): the caller's collectives
    // over host memory move the counts and the records (a gloo process group
    // rehearsing several ranks on one GPU, where RCCL refuses shared devices);
    // the routing, counts, offsets and receivers are this file's
    bool host = false;
    kb_group_host_transport ht{};
    std::vector<uint64_t> hsend, hrecv;  // staging, 8-B words
    std::vector<Rank> r;  // the ranks of this process
    uint32_t W = 0;       // record words
    uint32_t part = 0, n_parts = 1;
    int head = 0, tail = 0, inflight = 0;  // slots: next to send, next to receive
    Unit u[SLOTS];
    std::vector<uint64_t> last_C;  // counts of the last unit received or discarded
    // the sender thread: units' send stages in send order (RCCL calls on a
    // communicator stay in one order on every rank), so kb_group_send_async
    // returns at once and the caller's receive of the previous unit bins
    // while this one routes and exchanges
    std::thread th;
    std::mutex mu;
    std::condition_variable cv;
    std::deque<int> jobs;  // slots queued
    int running = 0;       // a job taken, not finished
    bool stop = false;
};

namespace {

// run f(i) for every local rank, one host thread each when there are several
// (kb_route_scatter and kb_finalize synchronise their context's stream: one
// thread would serialise the devices); the first failure is returned
template <typename F>
int for_ranks(kb_group* g, F&& f) {
    const int n = (int)g->r.size();
    if (n == 1) return f(0);
    std::vector<int> rc(n, KB_OK);
    std::vector<std::thread> th;
    for (int i = 0; i < n; i++)
        th.emplace_back([&, i] {
            rc[i] = f(i);
            if (rc[i]) g->r[i].err = kb_last_error();
        });
    for (auto& t : th) t.join();
    for (int i = 0; i < n; i++)
        if (rc[i]) return gfail(rc[i], "rank %d: %s", g->r[i].grank, g->r[i].err.c_str());
    return KB_OK;
}

int rank_init(kb_group* g, Rank& rk) {
    GHIP(hipSetDevice(rk.dev));
    kb_params p = g->p;
    p.device = rk.dev;
    GKB(kb_create(&p, &rk.recv));
    // the sender only scans and routes: first occurrences are the receiver's
    // (which then needs records in read order: plan/pack)
    rk.ordered = (g->p.flags & (KB_TRACK_FIRST | KB_ENGINE_TABLE)) != 0;
    p.flags &= ~KB_TRACK_FIRST;
    GKB(kb_create(&p, &rk.send));
    GHIP(hipStreamCreateWithFlags(&rk.xs, hipStreamNonBlocking));
    for (auto& e : rk.landed) GHIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    GHIP(hipEventCreateWithFlags(&rk.routed, hipEventDisableTiming));
    GHIP(hipHostMalloc((void**)&rk.h_counts, (size_t)g->G * (g->G + 1) * sizeof(uint64_t), hipHostMallocDefault));
    GHIP(rk.cdev.ensure((uint64_t)(g->G + 1) * (g->G + 1)));
    return KB_OK;
}

int group_init(kb_group* g) {
    for (auto& rk : g->r) {
        const int rc = rank_init(g, rk);
        if (rc) return rc;
    }
    GKB(kb_record_words(g->r[0].send, &g->W));
    return KB_OK;
}

void rank_free(Rank& rk) {
    (void)hipSetDevice(rk.dev);
    if (rk.xs) (void)hipStreamSynchronize(rk.xs);
    if (rk.comm) (void)rccl().CommDestroy(rk.comm);
    kb_destroy(rk.send);
    kb_destroy(rk.recv);
    for (auto& b : rk.regions) b.release();
    for (auto& b : rk.rbuf) b.release();
    rk.cdev.release();
    if (rk.h_counts) (void)hipHostFree(rk.h_counts);
    for (auto& e : rk.landed)
        if (e) (void)hipEventDestroy(e);
    if (rk.routed) (void)hipEventDestroy(rk.routed);
    if (rk.xs) (void)hipStreamDestroy(rk.xs);
}

// sender side of rank i: every unshipped read batch into slot s.  One pass
// (kb_route_scatter: destination regions of a learned capacity, records in no
// particular order -- the binned receivers order lists by read id), or, for
// receivers that number occurrences by arrival (first-occurrence tracking,
// the table engine), plan/pack: destination-major, read order.
int rank_route_body(kb_group* g, int i, int s);
int rank_route(kb_group* g, int i, int s) {
    Rank& rk = g->r[i];
    rk.route_rc = rank_route_body(g, i, s);
    rk.err = rk.route_rc ? kb_last_error() : "";
    return rk.route_rc;
}
int rank_route_body(kb_group* g, int i, int s) {
    Rank& rk = g->r[i];
    GHIP(hipSetDevice(rk.dev));
    // (the slot's last sends must be out before its regions are rewritten)
    GHIP(hipStreamWaitEvent((hipStream_t)kb_stream(rk.send), rk.landed[s], 0));
    const int G = g->G;
    const uint64_t W = g->W;
    uint64_t* cnt = rk.h_counts + (uint64_t)rk.grank * (G + 1);  // (this rank's row of C)
    std::vector<uint64_t>& off = rk.soff[s];
    off.assign((size_t)G, 0);
    if (!rk.ordered) {
        if (rk.cap == 0) rk.cap = rk.n_reads * 15 / (uint64_t)G + 4096;  // (~10 records per 150-bp read)
        for (int attempt = 0; attempt < 3; attempt++) {
            GHIP(rk.regions[s].ensure((uint64_t)G * rk.cap * W));
            const int rc = kb_route_scatter(rk.send, (uint32_t)G, rk.regions[s].p, rk.cap, cnt);
            if (rc == KB_OK) {
                // (the layout this call wrote: destination d at d * cap -- the
                // headroom raised below is the NEXT unit's; raising it first
                // pointed the exchange at the wrong records whenever a
                // destination came within 10 % + 1024 of the old cap)
                for (int d = 0; d < G; d++) off[d] = (uint64_t)d * rk.cap;
                const uint64_t mx = *std::max_element(cnt, cnt + G);
                rk.cap = std::max(rk.cap, mx + mx / 10 + 1024);
                return KB_OK;
            }
            if (rc == KB_EINVAL) break;  // (the one-pass sender does not apply: plan/pack)
            if (rc != KB_EOVERFLOW) return gfail(rc, "kb_route_scatter: %s", kb_last_error());
            const uint64_t mx = *std::max_element(cnt, cnt + G);
            rk.cap = mx + mx / 5 + 1024;
            if (attempt == 2) return gfail(KB_EDEVICE, "kb_route_scatter: region capacity not converging");
        }
        rk.ordered = true;
    }
    GKB(kb_route_plan(rk.send, (uint32_t)G, cnt));
    uint64_t tot = 0;
    for (int d = 0; d < G; d++) {
        off[d] = tot;
        tot += cnt[d];
    }
    GHIP(rk.regions[s].ensure(std::max<uint64_t>(tot, 1) * W));
    GKB(kb_route_pack(rk.send, rk.regions[s].p));
    return KB_OK;
}

// the counts matrix on every rank: RCCL all-gather of each rank's row, or
// (local transport) the rows are already in this process.  A row carries its
// rank's routing status after its G counts, so a rank whose routing failed
// still takes part in the all-gather and every rank returns the failure
// (an early return left the peers blocked in ncclAllGather)
int exchange_counts(kb_group* g, Unit& un) {
    const int G = g->G, RS = G + 1;
    un.C.assign((size_t)G * G, 0);
    for (auto& rk : g->r) rk.h_counts[(size_t)rk.grank * RS + G] = (uint64_t)(uint32_t)rk.route_rc;
    std::vector<uint64_t> rows((size_t)G * RS);
    if (g->local) {
        for (auto& rk : g->r)
            memcpy(&rows[(size_t)rk.grank * RS], rk.h_counts + (size_t)rk.grank * RS, RS * sizeof(uint64_t));
    } else if (g->host) {
        const Rank& rk = g->r[0];
        if (g->ht.allgather(g->ht.user, rk.h_counts + (size_t)rk.grank * RS, (uint64_t)RS, rows.data()))
            return gfail(KB_EDEVICE, "host transport: counts all-gather failed");
    } else {
        Rccl& R = rccl();
        for (auto& rk : g->r) {
            GHIP(hipSetDevice(rk.dev));
            GHIP(hipMemcpyAsync(rk.cdev.p, rk.h_counts + (size_t)rk.grank * RS, RS * sizeof(uint64_t),
                                hipMemcpyHostToDevice, rk.xs));
        }
        GNCCL(R.GroupStart());
        for (auto& rk : g->r)
            GNCCL(R.AllGather(rk.cdev.p, rk.cdev.p + RS, (size_t)RS, ncclUint64, rk.comm, rk.xs));
        GNCCL(R.GroupEnd());
        for (auto& rk : g->r) {
            GHIP(hipSetDevice(rk.dev));
            GHIP(hipMemcpyAsync(rk.h_counts, rk.cdev.p + RS, (size_t)G * RS * sizeof(uint64_t),
                                hipMemcpyDeviceToHost, rk.xs));
        }
        // (the sizes of the record sends are the host's to know: this is the
        // exchange's one host wait, on the group's sender thread)
        for (auto& rk : g->r) {
            GHIP(hipSetDevice(rk.dev));
            GHIP(hipStreamSynchronize(rk.xs));
        }
        memcpy(rows.data(), g->r[0].h_counts, rows.size() * sizeof(uint64_t));
        for (size_t k = 1; k < g->r.size(); k++)
            if (memcmp(rows.data(), g->r[k].h_counts, rows.size() * sizeof(uint64_t)))
                return gfail(KB_EDEVICE, "internal: ranks disagree on the record counts");
    }
    for (int src = 0; src < G; src++) {
        const uint64_t st = rows[(size_t)src * RS + G];
        if (st) {
            const Rank* mine = nullptr;
            for (auto& rk : g->r)
                if (rk.grank == src) mine = &rk;
            return gfail((int)st, "rank %d failed to route its records%s%s", src, mine ? ": " : " (peer)",
                         mine ? mine->err.c_str() : "");
        }
        memcpy(&un.C[(size_t)src * G], &rows[(size_t)src * RS], G * sizeof(uint64_t));
    }
    return KB_OK;
}

static uint64_t genv_u64(const char* k, uint64_t d) {
    const char* v = getenv(k);
    return v && *v ? strtoull(v, nullptr, 0) : d;
}

// the records: rank s's region for d -> rank d's receive slot, sources in
// rank order (received records concatenated by source rank)
int exchange_records(kb_group* g, Unit& un, int s) {
    const int G = g->G;
    const uint64_t W = g->W;
    for (auto& rk : g->r) {
        uint64_t tot = 0;
        for (int src = 0; src < G; src++) tot += un.C[(size_t)src * G + rk.grank];
        GHIP(hipSetDevice(rk.dev));
        // (the receive slot of the unit received two sends ago: its finalize
        // has returned, nothing references it now)
        GHIP(rk.rbuf[s].ensure(std::max<uint64_t>(tot, 1) * W));
        // (the regions were written on the sender's stream: the exchange
        // streams wait for them there, no host wait)
        GHIP(hipEventRecord(rk.routed, (hipStream_t)kb_stream(rk.send)));
    }
    for (auto& rk : g->r) {
        GHIP(hipSetDevice(rk.dev));
        if (g->local)  // (device copies read every local sender's regions)
            for (auto& src : g->r) GHIP(hipStreamWaitEvent(rk.xs, src.routed, 0));
        else
            GHIP(hipStreamWaitEvent(rk.xs, rk.routed, 0));
    }
    if (g->local) {
        for (auto& dst : g->r) {
            uint64_t off = 0;
            GHIP(hipSetDevice(dst.dev));
            for (int src = 0; src < G; src++) {
                const uint64_t n = un.C[(size_t)src * G + dst.grank];
                const Rank& sr = g->r[src];  // (local: every rank is here, in rank order)
                if (n)
                    GHIP(hipMemcpyAsync(dst.rbuf[s].p + off * W, sr.regions[s].p + sr.soff[s][dst.grank] * W,
                                        n * W * sizeof(uint64_t), hipMemcpyDeviceToDevice, dst.xs));
                off += n;
            }
        }
    } else if (g->host) {
        // the rank's region slices to the host (packed by destination), the
        // caller's all-to-all, the received records back to the receive slot
        Rank& rk = g->r[0];
        std::vector<uint64_t> sb(G), rb(G);
        uint64_t ns = 0, nr = 0;
        for (int peer = 0; peer < G; peer++) {
            sb[peer] = un.C[(size_t)rk.grank * G + peer] * W * sizeof(uint64_t);
            rb[peer] = un.C[(size_t)peer * G + rk.grank] * W * sizeof(uint64_t);
            ns += sb[peer] / 8;
            nr += rb[peer] / 8;
        }
        g->hsend.resize(std::max<uint64_t>(ns, 1));
        g->hrecv.resize(std::max<uint64_t>(nr, 1));
        GHIP(hipSetDevice(rk.dev));
        uint64_t o = 0;
        for (int peer = 0; peer < G; peer++) {
            if (sb[peer])
                GHIP(hipMemcpyAsync(g->hsend.data() + o, rk.regions[s].p + rk.soff[s][peer] * W, sb[peer],
                                    hipMemcpyDeviceToHost, rk.xs));
            o += sb[peer] / 8;
        }
        GHIP(hipStreamSynchronize(rk.xs));
        if (g->ht.alltoallv(g->ht.user, g->hsend.data(), sb.data(), g->hrecv.data(), rb.data()))
            return gfail(KB_EDEVICE, "host transport: record all-to-all failed");
        if (nr) GHIP(hipMemcpyAsync(rk.rbuf[s].p, g->hrecv.data(), nr * 8, hipMemcpyHostToDevice, rk.xs));
        // (the staging is reused by the next unit: the copy completes first)
        GHIP(hipStreamSynchronize(rk.xs));
    } else {
        // A rank's own records are a device copy.  Peer messages go in pieces
        // of at most XCHUNK words, matched in order on both sides: a one-rank
        // RCCL group's self send/recv of C4's pass (6 GB at 125 M reads)
        // delivered only about half of its records, the rest of the receive
        // slot left as it was -- every such record then read as a zero-length
        // TTTTTTT super-k-mer (one bucket of 129 M records, KB_ENOMEM)
        const uint64_t XCHUNK = genv_u64("KB_GROUP_CHUNK", 1ull << 25);  // 256 MB of records (words per piece)
        const bool self_rccl = genv_u64("KB_GROUP_SELF_RCCL", 0) != 0;  // (tests: the self copy by RCCL)
        const auto pieces = [&](uint64_t n, const auto& f) -> int {
            for (uint64_t o = 0; o < n;) {
                const uint64_t c = XCHUNK ? std::min<uint64_t>(n - o, XCHUNK) : n - o;
                if (const int rc = f(o, c)) return rc;
                o += c;
            }
            return KB_OK;
        };
        for (auto& rk : g->r) {
            const uint64_t n = un.C[(size_t)rk.grank * G + rk.grank];
            uint64_t off = 0;
            for (int src = 0; src < rk.grank; src++) off += un.C[(size_t)src * G + rk.grank];
            if (n && !self_rccl) {
                GHIP(hipSetDevice(rk.dev));
                GHIP(hipMemcpyAsync(rk.rbuf[s].p + off * W, rk.regions[s].p + rk.soff[s][rk.grank] * W,
                                    n * W * sizeof(uint64_t), hipMemcpyDeviceToDevice, rk.xs));
            }
        }
        Rccl& R = rccl();
        GNCCL(R.GroupStart());
        for (auto& rk : g->r) {
            uint64_t off = 0;
            for (int peer = 0; peer < G; peer++) {
                const uint64_t ns = un.C[(size_t)rk.grank * G + peer], nr = un.C[(size_t)peer * G + rk.grank];
                if (peer != rk.grank || self_rccl) {
                    const uint64_t* sp = rk.regions[s].p + rk.soff[s][peer] * W;
                    uint64_t* rp = rk.rbuf[s].p + off * W;
                    const int rc = pieces(ns * W, [&](uint64_t o, uint64_t c) -> int {
                        GNCCL(R.Send(sp + o, (size_t)c, ncclUint64, peer, rk.comm, rk.xs));
                        return KB_OK;
                    });
                    if (rc) return rc;
                    const int rc2 = pieces(nr * W, [&](uint64_t o, uint64_t c) -> int {
                        GNCCL(R.Recv(rp + o, (size_t)c, ncclUint64, peer, rk.comm, rk.xs));
                        return KB_OK;
                    });
                    if (rc2) return rc2;
                }
                off += nr;
            }
        }
        GNCCL(R.GroupEnd());
    }
    for (auto& rk : g->r) {
        GHIP(hipSetDevice(rk.dev));
        GHIP(hipEventRecord(rk.landed[s], rk.xs));
    }
    return KB_OK;
}

bool valid_local(kb_group* g, int i) { return g && i >= 0 && i < (int)g->r.size(); }

// one unit's send stage (the sender thread): every local rank routes, the
// counts (with each rank's routing status) go round, the records are sent
int send_stage(kb_group* g, int s) {
    Unit& un = g->u[s];
    (void)for_ranks(g, [&](int i) { return rank_route(g, i, s); });  // (failures travel with the counts)
    int rc = exchange_counts(g, un);
    if (!rc) rc = exchange_records(g, un, s);
    return rc;
}

void sender_loop(kb_group* g) {
    std::unique_lock<std::mutex> lk(g->mu);
    for (;;) {
        g->cv.wait(lk, [&] { return g->stop || !g->jobs.empty(); });
        if (g->jobs.empty()) return;  // (stop, nothing queued)
        const int s = g->jobs.front();
        g->jobs.pop_front();
        g->running++;
        lk.unlock();
        const int rc = send_stage(g, s);
        const std::string err = rc ? kb_last_error() : "";
        lk.lock();
        g->u[s].rc = rc;
        g->u[s].err = err;
        g->u[s].done = true;
        g->running--;
        g->cv.notify_all();
    }
}

// the sender thread idle: no unit routing (the senders' reads may change)
void wait_idle(kb_group* g) {
    std::unique_lock<std::mutex> lk(g->mu);
    g->cv.wait(lk, [&] { return g->jobs.empty() && g->running == 0; });
}

// the oldest unit's send stage finished; its outcome
int wait_unit(kb_group* g, int s) {
    std::unique_lock<std::mutex> lk(g->mu);
    g->cv.wait(lk, [&] { return g->u[s].done; });
    return g->u[s].rc;
}

int retire(kb_group* g, int s) {  // the oldest unit leaves (received or discarded)
    Unit& un = g->u[s];
    un.busy = false;
    g->last_C = un.C;
    g->tail = (s + 1) % SLOTS;
    g->inflight--;
    return KB_OK;
}

}  // namespace

// ---------------------------------------------------------------- C-ABI

extern "C" int kb_group_unique_id(void* out, size_t len) {
    if (!out || len < sizeof(ncclUniqueId)) return gfail(KB_EINVAL, "unique id needs %zu bytes", sizeof(ncclUniqueId));
    Rccl& R = rccl();
    if (!R.ok) return gfail(KB_EDEVICE, "RCCL unavailable: %s", R.why.c_str());
    ncclUniqueId id;
    GNCCL(R.GetUniqueId(&id));
    memcpy(out, &id, sizeof id);
    return KB_OK;
}

extern "C" int kb_group_create(const kb_params* p, int n_gpus, const int* devices, kb_group** out) {
    if (!p || !out || n_gpus < 1 || n_gpus > 64) return gfail(KB_EINVAL, "kb_group_create: bad arguments");
    *out = nullptr;
    kb_group* g = new kb_group();
    g->p = *p;
    g->G = n_gpus;
    g->r.resize(n_gpus);
    std::vector<int> devs(n_gpus);
    bool dup = false;
    for (int i = 0; i < n_gpus; i++) {
        devs[i] = devices ? devices[i] : i;
        for (int k = 0; k < i; k++) dup = dup || devs[k] == devs[i];
        g->r[i].dev = devs[i];
        g->r[i].grank = i;
    }
    // every rank in this process: RCCL communicators over distinct devices,
    // device copies for virtual shards (several ranks on one device) or on
    // request (KB_GROUP_TRANSPORT=local)
    const char* tr = getenv("KB_GROUP_TRANSPORT");
    g->local = dup || (tr && !strcmp(tr, "local"));
    int rc = group_init(g);
    if (!rc && !g->local) {
        Rccl& R = rccl();
        if (!R.ok) rc = gfail(KB_EDEVICE, "RCCL unavailable: %s", R.why.c_str());
        else {
            std::vector<ncclComm_t> comms(n_gpus);
            const ncclResult_t nr = R.CommInitAll(comms.data(), n_gpus, devs.data());
            if (nr != ncclSuccess) rc = gfail(KB_EDEVICE, "ncclCommInitAll: %s", R.GetErrorString(nr));
            else
                for (int i = 0; i < n_gpus; i++) g->r[i].comm = comms[i];
        }
    }
    if (rc) {
        const std::string e = kb_last_error();
        kb_group_destroy(g);
        return gfail(rc, "%s", e.c_str());
    }
    *out = g;
    return KB_OK;
}

extern "C" int kb_group_create_rank(const kb_params* p, int rank, int n_ranks, const void* unique_id, size_t len,
                                    kb_group** out) {
    if (!p || !out || !unique_id || len < sizeof(ncclUniqueId) || n_ranks < 1 || rank < 0 || rank >= n_ranks)
        return gfail(KB_EINVAL, "kb_group_create_rank: bad arguments");
    *out = nullptr;
    Rccl& R = rccl();
    if (!R.ok) return gfail(KB_EDEVICE, "RCCL unavailable: %s", R.why.c_str());
    kb_group* g = new kb_group();
    g->p = *p;
    g->G = n_ranks;
    g->r.resize(1);
    g->r[0].dev = p->device;
    g->r[0].grank = rank;
    int rc = group_init(g);
    if (!rc) {
        ncclUniqueId id;
        memcpy(&id, unique_id, sizeof id);
        (void)hipSetDevice(p->device);
        const ncclResult_t nr = R.CommInitRank(&g->r[0].comm, n_ranks, id, rank);
        if (nr != ncclSuccess) rc = gfail(KB_EDEVICE, "ncclCommInitRank: %s", R.GetErrorString(nr));
    }
    if (rc) {
        const std::string e = kb_last_error();
        kb_group_destroy(g);
        return gfail(rc, "%s", e.c_str());
    }
    *out = g;
    return KB_OK;
}

extern "C" int kb_group_create_rank_host(const kb_params* p, int rank, int n_ranks, const kb_group_host_transport* t,
                                         kb_group** out) {
    if (!p || !out || !t || !t->allgather || !t->alltoallv || n_ranks < 1 || rank < 0 || rank >= n_ranks)
        return gfail(KB_EINVAL, "kb_group_create_rank_host: bad arguments");
    *out = nullptr;
    kb_group* g = new kb_group();
    g->p = *p;
    g->G = n_ranks;
    g->host = true;
    g->ht = *t;
    g->r.resize(1);
    g->r[0].dev = p->device;
    g->r[0].grank = rank;
    const int rc = group_init(g);
    if (rc) {
        const std::string e = kb_last_error();
        kb_group_destroy(g);
        return gfail(rc, "%s", e.c_str());
    }
    *out = g;
    return KB_OK;
}

extern "C" void kb_group_destroy(kb_group* g) {
    if (!g) return;
    {
        std::lock_guard<std::mutex> lk(g->mu);
        g->stop = true;
        // units sent but never received or discarded (kbin.h: a program error):
        // the queued ones never start their collectives -- a peer that has
        // already gone would leave them blocked in the counts all-gather
        // (ADVICE r05); a stage already running is waited for
        if (g->inflight)
            fprintf(stderr, "kbin: kb_group_destroy with %d unit(s) in flight (receive or discard them first)\n",
                    g->inflight);
        for (const int s : g->jobs) {
            g->u[s].rc = KB_ESTATE;
            g->u[s].err = "group destroyed before the unit was sent";
            g->u[s].done = true;
        }
        g->jobs.clear();
    }
    g->cv.notify_all();
    if (g->th.joinable()) g->th.join();
    for (auto& rk : g->r) rank_free(rk);
    delete g;
}

extern "C" int kb_group_info(kb_group* g, int* n_ranks, int* n_local, int* rank0, int* transport) {
    if (!g) return gfail(KB_EINVAL, "null group");
    if (n_ranks) *n_ranks = g->G;
    if (n_local) *n_local = (int)g->r.size();
    if (rank0) *rank0 = g->r[0].grank;
    if (transport) *transport = g->local ? KB_TRANSPORT_LOCAL : g->host ? KB_TRANSPORT_HOST : KB_TRANSPORT_RCCL;
    return KB_OK;
}

extern "C" kb_ctx* kb_group_ctx(kb_group* g, int local) { return valid_local(g, local) ? g->r[local].recv : nullptr; }

extern "C" int kb_group_reset(kb_group* g) {
    if (!g) return gfail(KB_EINVAL, "null group");
    wait_idle(g);  // (a unit still routing reads the senders' batches)
    // (units in flight keep their records: the regions and receive slots are
    // the group's, only the senders' read batches are dropped)
    for (auto& rk : g->r) {
        GKB(kb_reset(rk.send));
        rk.n_reads = 0;
    }
    g->part = 0;
    g->n_parts = 1;
    return KB_OK;
}

extern "C" int kb_group_submit_ids(kb_group* g, int local, const char* bases, const uint32_t* lens, uint64_t n_reads,
                                   const int32_t* ids) {
    if (!valid_local(g, local)) return gfail(KB_EINVAL, "bad local rank %d", local);
    wait_idle(g);
    GKB(kb_submit_ids(g->r[local].send, bases, lens, n_reads, ids));
    g->r[local].n_reads += n_reads;
    return KB_OK;
}

extern "C" int kb_group_submit_packed_device(kb_group* g, int local, const uint64_t* d_words, const uint32_t* d_lens,
                                             uint64_t n_reads, uint32_t words_per_read, int32_t first_id) {
    if (!valid_local(g, local)) return gfail(KB_EINVAL, "bad local rank %d", local);
    wait_idle(g);
    GKB(kb_submit_packed_device(g->r[local].send, d_words, d_lens, n_reads, words_per_read, first_id));
    g->r[local].n_reads += n_reads;
    return KB_OK;
}

extern "C" int kb_group_set_partition(kb_group* g, uint32_t part, uint32_t n_parts) {
    if (!g) return gfail(KB_EINVAL, "null group");
    wait_idle(g);
    for (auto& rk : g->r) GKB(kb_set_partition(rk.send, part, n_parts));
    g->part = part;
    g->n_parts = n_parts;
    return KB_OK;
}

extern "C" int kb_group_send_async(kb_group* g) {
    if (!g) return gfail(KB_EINVAL, "null group");
    if (g->inflight == SLOTS) return gfail(KB_ESTATE, "kb_group_send: %d units in flight already", SLOTS);
    wait_idle(g);  // (the last unit's routing read the senders: done before this one's starts)
    const int s = g->head;
    Unit& un = g->u[s];
    un.busy = true;
    un.part = g->part;
    un.n_parts = g->n_parts;
    un.C.assign((size_t)g->G * g->G, 0);
    {
        std::lock_guard<std::mutex> lk(g->mu);
        un.done = false;
        un.rc = KB_OK;
        un.err.clear();
        g->jobs.push_back(s);
        if (!g->th.joinable()) g->th = std::thread(sender_loop, g);
    }
    g->cv.notify_all();
    g->head = (s + 1) % SLOTS;
    g->inflight++;
    return KB_OK;
}

extern "C" int kb_group_send(kb_group* g, uint64_t* h_counts) {
    int rc = kb_group_send_async(g);
    if (rc) return rc;
    const int s = (g->head + SLOTS - 1) % SLOTS;
    if ((rc = wait_unit(g, s))) {
        // (a failed unit leaves at once: nothing of it is in flight)
        const std::string e = g->u[s].err;
        g->head = s;
        g->u[s].busy = false;
        g->u[s].done = true;
        g->inflight--;
        return gfail(rc, "%s", e.c_str());
    }
    if (h_counts) memcpy(h_counts, g->u[s].C.data(), g->u[s].C.size() * sizeof(uint64_t));
    return KB_OK;
}

extern "C" int kb_group_unit_counts(kb_group* g, uint64_t* h_counts) {
    if (!g || !h_counts) return gfail(KB_EINVAL, "kb_group_unit_counts: bad arguments");
    if (g->last_C.empty()) return gfail(KB_ESTATE, "kb_group_unit_counts: no unit received yet");
    memcpy(h_counts, g->last_C.data(), g->last_C.size() * sizeof(uint64_t));
    return KB_OK;
}

extern "C" int kb_group_receive(kb_group* g, int prune) {
    if (!g) return gfail(KB_EINVAL, "null group");
    if (!g->inflight) return gfail(KB_ESTATE, "kb_group_receive: nothing sent");
    const int s = g->tail;
    Unit& un = g->u[s];
    const int G = g->G;
    if (const int src = wait_unit(g, s)) {
        const std::string e = un.err;
        retire(g, s);
        return gfail(src, "%s", e.c_str());
    }
    const int rc = for_ranks(g, [&](int i) -> int {
        Rank& rk = g->r[i];
        GHIP(hipSetDevice(rk.dev));
        GKB(kb_reset(rk.recv));
        if (un.n_parts > 1) GKB(kb_set_partition(rk.recv, un.part, un.n_parts));
        GHIP(hipStreamWaitEvent((hipStream_t)kb_stream(rk.recv), rk.landed[s], 0));
        uint64_t tot = 0;
        for (int src = 0; src < G; src++) tot += un.C[(size_t)src * G + rk.grank];
        if (getenv("KB_DEBUG") && atoi(getenv("KB_DEBUG")))
            fprintf(stderr, "[kb] group receive: rank %d, part %u/%u, %llu records\n", rk.grank, un.part, un.n_parts,
                    (unsigned long long)tot);
        if (tot) GKB(kb_submit_superkmers_device(rk.recv, rk.rbuf[s].p, tot));
        GKB(kb_finalize(rk.recv, prune));
        return KB_OK;
    });
    retire(g, s);
    return rc;
}

extern "C" int kb_group_discard(kb_group* g) {
    if (!g) return gfail(KB_EINVAL, "null group");
    if (!g->inflight) return gfail(KB_ESTATE, "kb_group_discard: nothing sent");
    const int s = g->tail;
    Unit& un = g->u[s];
    const int src = wait_unit(g, s);
    if (src) { // (kbin.h: _discard returns the unit's failure, as _receive does)
        const std::string e = un.err;
        retire(g, s);
        return gfail(src, "%s", e.c_str());
    }
    for (auto& rk : g->r) {
        GHIP(hipSetDevice(rk.dev));
        GHIP(hipEventSynchronize(rk.landed[s]));
    }
    retire(g, s);
    return KB_OK;
}

extern "C" int kb_group_finalize(kb_group* g, int prune) {
    const int rc = kb_group_send(g, nullptr);
    if (rc) return rc;
    return kb_group_receive(g, prune);
}
