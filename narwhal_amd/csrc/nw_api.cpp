// C-ABI host layer of libnwcrypto (include/nwcrypto.h): device memory, the key cache, per-call
// workspaces and streams, and the launch sequences.  No CPU compute path: every verdict and digest
// comes from the GPU.
//
// Concurrency model (the worker calls from 64 rayon threads,
// worker/src/processor.rs:75-79):
//   * the key cache (committee tables, basepoint comb) is shared state behind a reader/writer lock:
//     every verify call holds it shared while it enqueues; nw_committee_load holds it exclusive and
//     first waits for every in-flight call that may still read the tables;
//   * every call leases a Workspace from a pool: its own stream, scratch buffers, pinned staging
//     buffer and a completion event.  Host-buffer calls run on the workspace's stream and
//     synchronize it; ``_dev`` calls run on the caller's stream and leave the workspace "pending"
//     until its event completes — the next lease of that workspace waits on the event (stream
//     order, or a host wait before any buffer is reallocated), so scratch is never reused while a
//     kernel may still read it.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <random>
#include <shared_mutex>
#include <string>
#include <system_error>
#include <thread>
#include <unordered_map>
#include <vector>

#include "nw_build_id.h"
#include "nw_kernels.h"
#include "nw_msm.h"
#include "nw_point.h"

using namespace nw;

namespace {

thread_local std::string tl_last_error;

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) {
            hipError_t e = hipFree(p);
            if (e != hipSuccess) return e;
            p = nullptr;
            cap = 0;
        }
        size_t want = bytes < 4096 ? 4096 : bytes + bytes / 4;
        hipError_t e = hipMalloc(&p, want);
        if (e == hipSuccess) cap = want;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    template <typename T>
    T* as() const {
        return reinterpret_cast<T*>(p);
    }
};

// Pinned host staging buffer: one DMA per direction for the host-buffer entry points (pageable
// hipMemcpyAsync stages every call through a driver bounce buffer synchronously).
struct HostBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) {
            hipError_t e = hipHostFree(p);
            if (e != hipSuccess) return e;
            p = nullptr;
            cap = 0;
        }
        size_t want = bytes < 65536 ? 65536 : bytes + bytes / 4;
        hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
        if (e == hipSuccess) cap = want;
        return e;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
    }
    uint8_t* bytes() const { return reinterpret_cast<uint8_t*>(p); }
};

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// Key-cache map key: the 32 raw key bytes by value (no per-lookup allocation on the one-message
// paths), hashed with a per-process random seed so chosen keys cannot pile into one bucket.
struct Key32 {
    uint64_t w[4];
    explicit Key32(const uint8_t* p) { std::memcpy(w, p, 32); }
    bool operator==(const Key32& o) const {
        return w[0] == o.w[0] && w[1] == o.w[1] && w[2] == o.w[2] && w[3] == o.w[3];
    }
};
struct Key32Hash {
    static uint64_t seed() {
        static const uint64_t s = ((uint64_t)std::random_device{}() << 32) ^ std::random_device{}();
        return s;
    }
    static uint64_t mix(uint64_t x) {   // splitmix64 finalizer
        x ^= x >> 30;
        x *= 0xBF58476D1CE4E5B9ull;
        x ^= x >> 27;
        x *= 0x94D049BB133111EBull;
        return x ^ (x >> 31);
    }
    size_t operator()(const Key32& k) const {
        uint64_t h = seed();
        for (uint64_t v : k.w) h = mix(h ^ v);
        return (size_t)h;
    }
};

// Per-call scratch: one per concurrently executing call.
struct Workspace {
    hipStream_t stream = nullptr;   // stream of host-buffer calls
    hipEvent_t done = nullptr;      // recorded after the last enqueue that used these buffers
    hipStream_t last = nullptr;     // stream that event was recorded on
    bool pending = false;
    DevBuf w_sig, w_signer, w_keys, w_sig_cert, w_cert_first, w_cert_n, w_msg, w_msg_off, w_msg_len, w_flags,
        w_slow_count, w_slow_list, w_slow_slot, w_slow_buf, w_cert_ok, w_ok, w_misc, w_out, w_pbuf, w_pre, w_counts,
        w_cursor, w_perm, w_io, w_var, w_status, w_msm_ent, w_msm_dig, w_msm_zs, w_msm_meta, w_msm_bkt, w_msm_part,
        w_msm_wpart, w_pslow, w_cert_state, w_exact, w_pinfo;
    HostBuf h_io, h_meta;

    // Grow a buffer; a buffer that may still be read by a pending call is only freed after it.
    hipError_t ensure(DevBuf& b, size_t bytes) {
        if (bytes > b.cap && pending) {
            hipError_t e = hipEventSynchronize(done);
            if (e != hipSuccess) return e;
            pending = false;
        }
        return b.ensure(bytes);
    }
    void release_all() {
        for (DevBuf* b : {&w_sig, &w_signer, &w_keys, &w_sig_cert, &w_cert_first, &w_cert_n, &w_msg, &w_msg_off,
                          &w_msg_len, &w_flags, &w_slow_count, &w_slow_list, &w_slow_slot, &w_slow_buf, &w_cert_ok,
                          &w_ok, &w_misc, &w_out, &w_pbuf, &w_pre, &w_counts, &w_cursor, &w_perm, &w_io, &w_var,
                          &w_status, &w_msm_ent, &w_msm_dig, &w_msm_zs, &w_msm_meta, &w_msm_bkt, &w_msm_part,
                          &w_msm_wpart, &w_pslow, &w_cert_state, &w_exact, &w_pinfo})
            b->release();
        h_io.release();
        h_meta.release();
    }
};

constexpr size_t kMaxWorkspaces = 64;   // one per concurrently calling thread (the worker's 64)
// Asynchronous digest jobs hold a workspace from submit to nw_job_wait; past this many unwaited jobs
// a submit fails at once (NW_ERR_NOMEM) instead of blocking on a pool that only those jobs' own
// waits could refill.  The other half of the pool stays for synchronous calls.
constexpr int kMaxAsyncJobs = (int)kMaxWorkspaces / 2;

}  // namespace

struct nw_ctx {
    int device = 0;
    hipStream_t stream = nullptr;   // administrative stream: basepoint table, committee loads
    uint32_t finish_k = 0;          // k_finish signatures per lane (0: adaptive, finish_k_for)
    // key cache (shared by all calls; guarded by keys_mu)
    std::shared_mutex keys_mu;
    uint32_t* d_btab = nullptr;
    size_t max_keys = 0;          // 0: derived from the HBM budget once the window is fixed
    bool max_keys_user = false;
    int key_window = 0;           // 0: not yet decided (first load)
    bool committee_mode = false;  // nw_opts.key_window == -1
    bool key_reserve = false;     // committee mode + max_keys: the first load allocates max_keys slots
    bool budget_fixed = false;    // window, max_keys and reservation decided (first load with keys)
    size_t key_words = 0;         // u32 words per key-cache slot (T+, and T- when key_negtab)
    bool key_negtab = false;      // each key table followed by its negated copy (k_verify: no negation)
    uint32_t opt_flags = 0;       // nw_opts.flags (NW_OPT_*)
    size_t nkeys = 0, key_cap = 0;
    uint32_t* d_keys_raw = nullptr;
    uint32_t* d_key_info = nullptr;
    uint32_t* d_stake = nullptr;
    uint32_t* d_key_tab = nullptr;
    std::unordered_map<Key32, uint32_t, Key32Hash> slot_of;
    std::vector<uint32_t> h_stake;
    DevBuf w_bases;               // committee-load scratch (exclusive lock)
    // workspace pool
    std::mutex pool_mu;
    std::condition_variable pool_cv;
    std::vector<std::unique_ptr<Workspace>> pool;
    std::vector<Workspace*> free_ws;
    std::atomic<int> async_jobs{0};   // unwaited nw_sha512_many_async jobs (<= kMaxAsyncJobs)
    // measurement: (start, stop) event pairs around k_verify launches
    std::mutex prof_mu;
    bool prof_on = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> prof_events;
    size_t prof_used = 0;
    uint64_t prof_sigs = 0;
};

namespace {

uint32_t finish_k_for(const nw_ctx* ctx, size_t n) {
    if (ctx->finish_k) return ctx->finish_k;
    // k_finish<ONE> up to one lane per SIMD slot (256 CUs x 4 SIMDs x 64); above, the chunked kernel
    // (four waves per SIMD) with the fewest signatures per lane that still fits the chip in one round
    const size_t one_max = 256 * 4 * 64, lanes = one_max * 4;
    if (n <= one_max) return 1;
    const size_t k = (n + lanes - 1) / lanes;
    return k < 2 ? 2u : (k > (size_t)FINISH_K ? (uint32_t)FINISH_K : (uint32_t)k);
}

// Diagnostics are per calling thread (a context is shared by many threads).
void set_error(nw_ctx*, const std::string& msg) { tl_last_error = msg; }

int fail(nw_ctx* c, hipError_t e, const char* what) {
    set_error(c, std::string(what) + ": " + hipGetErrorString(e));
    return e == hipErrorOutOfMemory ? NW_ERR_NOMEM : NW_ERR_DEVICE;
}

#define NW_TRY(expr, what)                              \
    do {                                                \
        hipError_t e_ = (expr);                         \
        if (e_ != hipSuccess) return fail(ctx, e_, what); \
    } while (0)

// Lease of a workspace for one call.  ``bind(st)`` orders the call after the workspace's previous
// user; ``finish(st)`` records the completion event (kept pending for asynchronous calls).  A
// host-buffer call that fails after enqueueing synchronizes its stream on release, so no DMA from
// its pinned buffer and no kernel on its scratch outlives the call.
//
// Which free workspace a call gets: one whose last work was on the call's own stream (stream order
// already serializes them), else one with no work in flight, else a new one while the pool is below
// kMaxWorkspaces.  So device-buffer calls alternating over two streams (one batch's k_finish and
// slow path under the next batch's k_verify) run on two workspaces and never wait for each other;
// only a full pool falls back to the most recently freed workspace and its completion event.
class Lease {
public:
    // pinned_hint: bytes of pinned staging the call will need; an idle workspace that already has
    // them is preferred (growing a pinned buffer costs ~0.1 s per GB of pinning, and the first DMAs
    // from new pinned pages stall: a 1,250-batch worker window on a workspace grown mid-run ran at
    // half the rate, r04w).
    explicit Lease(nw_ctx* ctx, hipStream_t st = nullptr, size_t pinned_hint = 0) : ctx_(ctx) {
        std::unique_lock<std::mutex> g(ctx->pool_mu);
        for (;;) {
            auto& fr = ctx->free_ws;
            if (!fr.empty()) {
                size_t pick = fr.size();
                for (size_t i = fr.size(); i-- > 0 && pick == fr.size();)
                    if (fr[i]->pending && st && fr[i]->last == st) pick = i;
                auto idle = [&](size_t i) { return !fr[i]->pending || hipEventQuery(fr[i]->done) == hipSuccess; };
                if (pinned_hint)
                    for (size_t i = fr.size(); i-- > 0 && pick == fr.size();)
                        if (fr[i]->h_io.cap >= pinned_hint && idle(i)) pick = i;
                for (size_t i = fr.size(); i-- > 0 && pick == fr.size();)
                    if (idle(i)) pick = i;
                if (pick == fr.size() && ctx->pool.size() < kMaxWorkspaces) break;   // all busy: a new one
                if (pick == fr.size()) pick = fr.size() - 1;
                ws_ = fr[pick];
                fr.erase(fr.begin() + (ptrdiff_t)pick);
                return;
            }
            if (ctx->pool.size() < kMaxWorkspaces) break;
            ctx->pool_cv.wait(g);
        }
        auto w = std::make_unique<Workspace>();
        if (hipStreamCreateWithFlags(&w->stream, hipStreamNonBlocking) != hipSuccess) return;
        if (hipEventCreateWithFlags(&w->done, hipEventDisableTiming) != hipSuccess) {
            (void)hipStreamDestroy(w->stream);
            return;
        }
        ws_ = w.get();
        ctx->pool.push_back(std::move(w));
    }
    ~Lease() {
        if (!ws_) return;
        const bool drain = sync_on_release_ && stream_;
        if (drain) (void)hipStreamSynchronize(stream_);
        std::lock_guard<std::mutex> g(ctx_->pool_mu);
        if (drain) ws_->pending = false;
        ctx_->free_ws.push_back(ws_);
        ctx_->pool_cv.notify_one();
    }
    Workspace* ws() const { return ws_; }
    hipError_t bind(hipStream_t st, bool sync_on_release) {
        stream_ = st;
        sync_on_release_ = sync_on_release;
        if (ws_->pending && ws_->last != st) return hipStreamWaitEvent(st, ws_->done, 0);
        return hipSuccess;
    }
    hipError_t finish() {
        hipError_t e = hipEventRecord(ws_->done, stream_);
        if (e == hipSuccess) {
            std::lock_guard<std::mutex> g(ctx_->pool_mu);
            ws_->pending = true;
            ws_->last = stream_;
        }
        return e;
    }
    // a host-buffer call that completed: its stream is idle
    void synced() {
        std::lock_guard<std::mutex> g(ctx_->pool_mu);   // drain_all reads pending under pool_mu
        ws_->pending = false;
        sync_on_release_ = false;
    }

private:
    nw_ctx* ctx_;
    Workspace* ws_ = nullptr;
    hipStream_t stream_ = nullptr;
    bool sync_on_release_ = false;
};

}  // namespace

// An asynchronous host-buffer call in flight (nw_sha512_many_async): its workspace lease, the
// caller's output and where the digests land in the workspace's pinned buffer.
struct nw_job {
    std::unique_ptr<Lease> lease;
    uint8_t* out = nullptr;
    size_t n = 0;
    size_t o_out = 0;
    std::atomic<int>* inflight = nullptr;   // the context's async job count (released with the job)
    ~nw_job() {
        lease.reset();
        if (inflight) inflight->fetch_sub(1);
    }
};

namespace {

// Wait for every call that may still read the key tables (exclusive key lock held).  Every
// verification lease is taken under the shared key lock, so none is live here.  Asynchronous
// digest jobs (nw_sha512_many_async) hold their lease WITHOUT the key lock, so one may be live: it
// reads no key table, its completion event is only re-recorded by its own submit, and every write
// of ``pending`` (Lease::finish / synced / release) happens under pool_mu, as these reads do.
int drain_all(nw_ctx* ctx) {
    std::lock_guard<std::mutex> g(ctx->pool_mu);
    for (auto& w : ctx->pool)
        if (w->pending) {
            NW_TRY(hipEventSynchronize(w->done), "drain");
            w->pending = false;
        }
    return NW_OK;
}

// Basepoint encoding (y = 4/5, x even).
const uint8_t kBaseEnc[32] = {0x58, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66,
                              0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66,
                              0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66};

// k_finish signatures per lane: adaptive (finish_k_for); variant builds for A/B runs may pin it with
// -DNW_FK_FIXED=k (tools/build_variants.sh).  Measured on MI355X: splitting a batch into chunks so
// k_finish of one chunk overlaps k_verify of the next on a second stream was slower (623 vs 712 M
// sigs/s at C2: the co-running k_finish waves take VGPR slots from the VALU-bound k_verify and every
// chunk pays a tail), so a batch is one k_verify + one k_finish.
#ifndef NW_FK_FIXED
#define NW_FK_FIXED 0
#endif
static_assert(NW_FK_FIXED >= 0 && NW_FK_FIXED <= FINISH_K, "NW_FK_FIXED: 0 (adaptive) or 1..FINISH_K");
// Signer grouping on (1, release) or off (0: variant builds for the A/B of the grouping itself).
#ifndef NW_GROUP_SIGNERS
#define NW_GROUP_SIGNERS 1
#endif

// Signatures per k_finish lane for a launch of n: just enough that the lanes fit one wave per SIMD
// (256 CUs x 4 SIMDs x 64 lanes), because below that the kernel is bound by the serial
// prefix-product chain + inversion of each lane, not by the inversion count.  A single
// certificate (67 .. 6,667 signatures) gets one signature per lane: one inversion per signature,
// no chain; C2's million signatures get 16 per lane.
uint32_t finish_k_for(const nw_ctx* ctx, size_t n);

// HBM for key tables: what the device has free at the first committee load (after this context's
// basepoint table and whatever other contexts or processes on the GPU hold), less a reserve for call
// workspaces.  A node may run its primary and a worker on one GPU; a fixed share per context could
// not see the other.
constexpr size_t kWorkspaceReserve = 16ull << 30;   // at least this much stays free for workspaces
size_t key_budget(nw_ctx* ctx) {
    size_t free_b = 0, total_b = 0;
    if (hipSetDevice(ctx->device) != hipSuccess || hipMemGetInfo(&free_b, &total_b) != hipSuccess || total_b == 0)
        return 0;
    const size_t reserve = std::max(kWorkspaceReserve, total_b / 16);
    return free_b > reserve ? free_b - reserve : 0;
}
// Group signatures by signer (key-table locality) above this batch size, and only when keys repeat
// (at least kGroupMinSigsPerKey signatures per cached key on average): the worker's load (62,500
// signatures over 100,000 keys, each key at most once) gains nothing from the order and would pay
// the 100,000-slot scan (0.16 ms of a 0.47 ms batch, profiles/r02/kernel_stats_w_r02.csv).
constexpr size_t kGroupMinSigs = 16384;
constexpr size_t kGroupMinSigsPerKey = 4;

// Key comb window, fixed at the first load.  Auto (0): a conservative choice that leaves room for
// keys added later.  Committee mode (-1): take the widest window (fewest additions per signature)
// whose tables fit the budget for ``n`` keys times ``headroom``:
//   - without nw_opts.max_keys the first load IS the committee, with 25% headroom for later keys;
//   - with nw_opts.max_keys the caller has declared every key it will load (the worker's two
//     Processors, 2 x 100,000 simulation keys, worker/src/processor.rs:46-58 and worker.rs:182,228):
//     sized for exactly that many, and the cache is allocated for all of them at the first load
//     (grow_keys), so the second Processor's load appends without a growth copy.
int committee_window(size_t n, double headroom, size_t budget) {
    for (int w : {20, 16, 13, 12, 9}) {
        const double need = headroom * (double)n * (double)comb_words(w) * 4.0;
        if (need <= (double)budget) return w;
    }
    return 8;
}

void fix_window(nw_ctx* ctx, size_t first_load) {
    const size_t budget = key_budget(ctx);
    const bool auto_window = ctx->key_window == 0;
    if (ctx->key_window == -1)
        ctx->key_window = ctx->max_keys_user ? committee_window(std::max(ctx->max_keys, first_load), 1.0, budget)
                                             : committee_window(first_load, 1.25, budget);
    if (ctx->key_window == 0) ctx->key_window = first_load <= 384 ? 16 : (first_load <= 12288 ? 12 : 8);
    // Negated copies (T-) of the key tables when twice the tables still fit the budget for the keys
    // this context is sized for: k_verify's key pass then needs no conditional negation (7% of its
    // time at C2).  A large worker cache keeps the wider window instead (2 fewer comb positions are
    // worth more than the negation).  NW_OPT_NO_KEY_NEGTAB turns it off.
    // Sized for: the declared max_keys, else the first load with 25% headroom (committee mode, or a
    // window the caller chose).  An automatic window (nw_opts.key_window 0) is for callers that add
    // keys over time with no declared bound: it never takes T-, whose doubled tables would halve the
    // capacity max_keys allows below (the choice is permanent for the context).
    const double sized = ctx->max_keys_user ? (double)std::max(ctx->max_keys, first_load) : (double)first_load * 1.25;
    ctx->key_negtab = !(ctx->opt_flags & NW_OPT_NO_KEY_NEGTAB) && !auto_window &&
                      2.0 * sized * (double)comb_words(ctx->key_window) * 4.0 <= (double)budget;
    ctx->key_words = comb_words(ctx->key_window) * (ctx->key_negtab ? 2 : 1);
    ctx->key_reserve = ctx->max_keys_user && ctx->committee_mode;
    ctx->budget_fixed = true;
    if (!ctx->max_keys_user) ctx->max_keys = budget / (ctx->key_words * 4);
}

int grow_keys(nw_ctx* ctx, size_t need) {
    if (need <= ctx->key_cap) return NW_OK;
    if (need > ctx->max_keys) {
        set_error(ctx, "key cache capacity exceeded (nw_opts.max_keys, or the HBM free at the first load)");
        return NW_ERR_NOMEM;
    }
    // The first load sizes the cache to its keys (rounded up to 64): in committee mode it IS the
    // committee, and doubling from 64 would reserve up to 2x the tables (16,384 W13 tables = 172 GB
    // for a 10,000-key committee, against 105 GB used).  Later loads grow it by doubling.
    size_t cap = ctx->key_cap ? ctx->key_cap : (ctx->key_reserve ? ctx->max_keys : (need + 63) / 64 * 64);
    while (cap < need) cap *= 2;
    if (cap > ctx->max_keys) cap = ctx->max_keys;
    uint32_t *raw = nullptr, *info = nullptr, *stake = nullptr, *tab = nullptr;
    auto cleanup = [&]() {
        for (uint32_t* p : {raw, info, stake, tab})
            if (p) (void)hipFree(p);
    };
    hipError_t e = hipMalloc(&raw, cap * 32);
    if (e == hipSuccess) e = hipMalloc(&info, cap * 4);
    if (e == hipSuccess) e = hipMalloc(&stake, cap * 4);
    if (e == hipSuccess) e = hipMalloc(&tab, cap * ctx->key_words * 4);
    if (e == hipSuccess && ctx->nkeys) {
        e = hipMemcpyAsync(raw, ctx->d_keys_raw, ctx->nkeys * 32, hipMemcpyDeviceToDevice, ctx->stream);
        if (e == hipSuccess)
            e = hipMemcpyAsync(info, ctx->d_key_info, ctx->nkeys * 4, hipMemcpyDeviceToDevice, ctx->stream);
        if (e == hipSuccess)
            e = hipMemcpyAsync(stake, ctx->d_stake, ctx->nkeys * 4, hipMemcpyDeviceToDevice, ctx->stream);
        if (e == hipSuccess)
            e = hipMemcpyAsync(tab, ctx->d_key_tab, ctx->nkeys * ctx->key_words * 4, hipMemcpyDeviceToDevice,
                               ctx->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    }
    if (e != hipSuccess) {
        (void)hipStreamSynchronize(ctx->stream);
        cleanup();
        return fail(ctx, e, "grow key cache");
    }
    for (uint32_t* p : {ctx->d_keys_raw, ctx->d_key_info, ctx->d_stake, ctx->d_key_tab})
        if (p) (void)hipFree(p);
    ctx->d_keys_raw = raw;
    ctx->d_key_info = info;
    ctx->d_stake = stake;
    ctx->d_key_tab = tab;
    ctx->key_cap = cap;
    return NW_OK;
}

// Build tables for nk keys whose raw bytes are already at d_raw (administrative stream).
int build_keys(nw_ctx* ctx, uint32_t* d_raw, uint32_t* d_info, uint32_t* d_tab, size_t nk, int window, size_t stride,
               bool negtab) {
    // keys per launch: bounds the bases scratch and keeps a launch near 16M chunk threads
    const size_t chunk = window >= 24 ? 1 : (window == 20 ? 16 : (window == 16 ? 256 : 4096));
    for (size_t s = 0; s < nk; s += chunk) {
        const size_t m = nk - s < chunk ? nk - s : chunk;
        if (m * comb_pos(window) * 40 * 4 > ctx->w_bases.cap) NW_TRY(hipStreamSynchronize(ctx->stream), "sync");
        NW_TRY(ctx->w_bases.ensure(m * comb_pos(window) * 40 * 4), "hipMalloc(bases)");
        NW_TRY(launch_key_prep((uint32_t)m, d_raw + s * 8, d_info + s, ctx->w_bases.as<uint32_t>(), d_tab + s * stride,
                               stride, negtab, window, ctx->stream),
               "k_key_prep/k_comb_build");
    }
    return NW_OK;
}

// Slots of keys already in the cache (shared lock held).  Returns true when every key is cached.
bool lookup_slots(nw_ctx* ctx, const uint8_t (*pk)[32], size_t n, uint32_t* slots) {
    for (size_t i = 0; i < n; ++i) {
        auto it = ctx->slot_of.find(Key32(pk[i]));
        if (it == ctx->slot_of.end()) return false;
        slots[i] = it->second;
    }
    return true;
}

// Map keys to cache slots, loading unknown keys (table build on the GPU).  Exclusive lock held.
int ensure_slots(nw_ctx* ctx, const uint8_t (*pk)[32], const uint32_t* stake, size_t n, uint32_t* slots) {
    std::vector<uint8_t> new_raw;
    std::vector<uint32_t> new_stake;
    std::vector<std::pair<uint32_t, uint32_t>> refresh;   // (slot, stake) of keys already cached
    std::unordered_map<Key32, uint32_t, Key32Hash> pending;
    for (size_t i = 0; i < n; ++i) {
        const Key32 k(pk[i]);
        auto it = ctx->slot_of.find(k);
        if (it != ctx->slot_of.end()) {
            slots[i] = it->second;
            // only a changed stake is a refresh: an unchanged reload must not drain every in-flight call
            if (stake && ctx->h_stake[it->second] != stake[i]) refresh.emplace_back(it->second, stake[i]);
            continue;
        }
        auto pit = pending.find(k);
        if (pit != pending.end()) {
            slots[i] = pit->second;
            if (stake) new_stake[pit->second - ctx->nkeys] = stake[i];
            continue;
        }
        const uint32_t slot = (uint32_t)(ctx->nkeys + pending.size());
        pending.emplace(k, slot);
        slots[i] = slot;
        new_raw.insert(new_raw.end(), pk[i], pk[i] + 32);
        new_stake.push_back(stake ? stake[i] : 0u);
    }
    const size_t add = pending.size();
    if (add == 0 && refresh.empty()) return NW_OK;
    int rc = drain_all(ctx);   // nothing in flight may read the tables or the stakes we change
    if (rc != NW_OK) return rc;
    if (add && !ctx->budget_fixed) fix_window(ctx, add);
    if (add) {
        rc = grow_keys(ctx, ctx->nkeys + add);
        if (rc != NW_OK) return rc;
        const size_t k0 = ctx->nkeys;
        NW_TRY(hipMemcpyAsync(ctx->d_keys_raw + k0 * 8, new_raw.data(), add * 32, hipMemcpyHostToDevice, ctx->stream),
               "H2D keys");
        rc = build_keys(ctx, ctx->d_keys_raw + k0 * 8, ctx->d_key_info + k0, ctx->d_key_tab + k0 * ctx->key_words,
                        add, ctx->key_window, ctx->key_words, ctx->key_negtab);
        if (rc != NW_OK) {
            (void)hipStreamSynchronize(ctx->stream);
            return rc;
        }
        NW_TRY(hipStreamSynchronize(ctx->stream), "sync(key tables)");
    }
    // the host stake table changes only once the tables are built
    std::vector<uint32_t> hs = ctx->h_stake;
    hs.insert(hs.end(), new_stake.begin(), new_stake.end());
    for (auto& r : refresh) hs[r.first] = r.second;
    NW_TRY(hipMemcpyAsync(ctx->d_stake, hs.data(), hs.size() * 4, hipMemcpyHostToDevice, ctx->stream), "H2D stake");
    NW_TRY(hipStreamSynchronize(ctx->stream), "sync(committee)");
    for (auto& kv : pending) ctx->slot_of.emplace(kv.first, kv.second);
    ctx->nkeys += add;
    ctx->h_stake.swap(hs);
    return NW_OK;
}

// Preamble state a small host-buffer call uploads with its inputs (one DMA), so the batch starts
// with no preamble kernels: the vote -> certificate map (host-expanded), the zeroed slow-path
// counter and the zeroed per-certificate exact-path state.
struct PreStaged {
    uint32_t* sig_cert;     // [nsigs + 1]
    uint32_t* zero4;        // [4]
    uint32_t* cert_state;   // [ncerts]
};
// Calls below this many signatures (and whose staged bytes fit kSmallCallBytes) use PreStaged:
// the signer grouping (k_expand_count's histogram) only runs from kGroupMinSigs up.
constexpr size_t kStagedMaxSigs = 16384;
static_assert(kStagedMaxSigs <= kGroupMinSigs, "staged calls never group");

// Certificate / batch vote ranges must be pairwise disjoint: a vote belongs to at most one
// certificate (its coefficient z and its exact-path term are keyed by that certificate).  Empty
// ranges never overlap anything.
bool ranges_disjoint(const uint32_t* first, const uint32_t* nv, size_t n) {
    std::vector<std::pair<uint64_t, uint64_t>> r;
    r.reserve(n);
    for (size_t c = 0; c < n; ++c)
        if (nv[c]) r.emplace_back(first[c], (uint64_t)first[c] + nv[c]);
    std::sort(r.begin(), r.end());
    for (size_t k = 1; k < r.size(); ++k)
        if (r[k].first < r[k - 1].second) return false;
    return true;
}

// Bytes of the PreStaged block for a call (256-B aligned segments).
size_t prestaged_bytes(size_t nsigs, size_t ncerts) {
    return align256((nsigs + 1) * 4) + 256 + align256(ncerts * 4 + 4);
}

// Fill the PreStaged block at h (host staging) and point pre at the same offsets from d.
void prestage(uint8_t* h, uint8_t* d, const uint32_t* first, const uint32_t* nv, size_t ncerts, size_t nsigs,
              PreStaged& pre) {
    const size_t o_sc = 0, o_z = align256((nsigs + 1) * 4), o_cs = o_z + 256;
    uint32_t* sc = reinterpret_cast<uint32_t*>(h + o_sc);
    std::memset(h, 0, prestaged_bytes(nsigs, ncerts));
    std::memset(h + o_sc, 0xFF, (nsigs + 1) * 4);   // NO_CERT: votes outside every range
    for (size_t c = 0; c < ncerts; ++c) {   // host-validated ranges: inside [0, nsigs), disjoint
        const size_t f = first[c], e = f + nv[c];
        for (size_t v = f; v < e; ++v) sc[v] = (uint32_t)c;
    }
    pre.sig_cert = reinterpret_cast<uint32_t*>(d + o_sc);
    pre.zero4 = reinterpret_cast<uint32_t*>(d + o_z);
    pre.cert_state = reinterpret_cast<uint32_t*>(d + o_cs);
}

// Enqueue the certificate pipeline on device buffers (shared key lock held, workspace bound to st).
// With ``pre`` the preamble state is already in device memory (small host-buffer calls).  A strict
// call's verdict bytes (d_sig_ok, batch_mode 0) come straight from k_finish.
int enqueue_certs(nw_ctx* ctx, Workspace* ws, size_t ncerts, const uint32_t* d_first, const uint32_t* d_nv,
                  size_t nsigs, const uint8_t* d_sig, const uint32_t* d_signer, int msgmode, const uint8_t* d_msg32,
                  const uint8_t* d_msg_base, const uint64_t* d_msg_off, const uint64_t* d_msg_len,
                  const uint8_t* zseed, uint64_t cert_base, uint32_t batch_mode, uint8_t* d_cert_ok,
                  uint32_t* d_flags_user, uint64_t* d_stake_out, hipStream_t st, uint8_t* d_sig_ok = nullptr,
                  uint32_t* d_status = nullptr, const PreStaged* pre = nullptr, bool sync_check = false) {
    uint32_t* d_flags = d_flags_user;
    if (!d_flags) {
        NW_TRY(ws->ensure(ws->w_flags, nsigs * 4 + 4), "ws flags");
        d_flags = ws->w_flags.as<uint32_t>();
    }
    NW_TRY(ws->ensure(ws->w_sig_cert, nsigs * 4 + 4), "ws sig_cert");
    NW_TRY(ws->ensure(ws->w_slow_count, 16), "ws slow_count");
    NW_TRY(ws->ensure(ws->w_slow_list, nsigs * 4 + 4), "ws slow_list");
    NW_TRY(ws->ensure(ws->w_slow_slot, nsigs * 4 + 4), "ws slow_slot");
    if (batch_mode) {
        NW_TRY(ws->ensure(ws->w_slow_buf, nsigs * (size_t)SLOW_WORDS * 4 + 4), "ws slow_buf");
        NW_TRY(ws->ensure(ws->w_pslow, nsigs * (size_t)160 + 16), "ws pslow");
        NW_TRY(ws->ensure(ws->w_cert_state, ncerts * 4 + 16), "ws cert_state");
        NW_TRY(ws->ensure(ws->w_exact, ncerts * 4 + 16), "ws exact list");
    }
    NW_TRY(ws->ensure(ws->w_pbuf, nsigs * (size_t)PBUF_WORDS * 4 + 16), "ws pbuf");
    NW_TRY(ws->ensure(ws->w_pre, nsigs * 40 + 16), "ws pre");
    // signer grouping (device counting sort) when keys repeat
    const bool group = NW_GROUP_SIGNERS && !pre && nsigs >= kGroupMinSigs && ctx->nkeys > 1 &&
                       nsigs >= kGroupMinSigsPerKey * ctx->nkeys;
    if (group) {
        NW_TRY(ws->ensure(ws->w_counts, ctx->nkeys * 4 + 16), "ws counts");
        NW_TRY(ws->ensure(ws->w_cursor, ctx->nkeys * 4 + 16), "ws cursor");
        NW_TRY(ws->ensure(ws->w_perm, nsigs * 4 + 16), "ws perm");
        NW_TRY(ws->ensure(ws->w_pinfo, nsigs * 8 + 16), "ws pinfo");
    }
    uint32_t* sig_cert = pre ? pre->sig_cert : ws->w_sig_cert.as<uint32_t>();
    uint32_t* slow_count = pre ? pre->zero4 : ws->w_slow_count.as<uint32_t>();
    uint32_t* cert_state = !batch_mode ? nullptr : (pre ? pre->cert_state : ws->w_cert_state.as<uint32_t>());
    if (!pre) {
        // Preamble in two launches: sig_cert = NO_CERT, zero the slot counts, the slow-path counter,
        // the certificate states and the status word; expand certificates; histogram signer slots;
        // check the device inputs into the status word.  sync_check: the call waits for that check
        // and returns NW_ERR_ARG before anything else is enqueued.
        if (sync_check) {
            NW_TRY(ws->ensure(ws->w_status, 16), "ws status");
            d_status = ws->w_status.as<uint32_t>();
        }
        NW_TRY(launch_prep_expand((uint32_t)ncerts, (uint32_t)nsigs, (uint32_t)ctx->nkeys, d_first, d_nv, d_signer,
                                  sig_cert, slow_count, group ? ws->w_counts.as<uint32_t>() : nullptr, d_status,
                                  cert_state, st),
               "k_prep_certs / k_expand_count");
        if (sync_check) {
            NW_TRY(ws->h_io.ensure(16), "pinned status");
            NW_TRY(hipMemcpyAsync(ws->h_io.p, d_status, 4, hipMemcpyDeviceToHost, st), "D2H status");
            NW_TRY(hipStreamSynchronize(st), "sync(status)");
            uint32_t sv = 0;
            std::memcpy(&sv, ws->h_io.p, 4);
            if (sv != 0) {
                set_error(ctx, "nw_verify_certs_dev: vote range past nsigs, overlapping vote ranges, or signer slot "
                               "outside the key cache");
                return NW_ERR_ARG;
            }
        }
    }

    VerifyParams vp{};
    vp.n = (uint32_t)nsigs;
    vp.batch_mode = batch_mode;
    vp.sig = d_sig;
    vp.signer = d_signer;
    vp.sig_cert = sig_cert;
    vp.cert_first = d_first;
    vp.cert_msg = d_msg32;
    vp.msg_base = d_msg_base;
    vp.msg_off = d_msg_off;
    vp.msg_len = d_msg_len;
    vp.cert_base = cert_base;
    vp.keys_raw = ctx->d_keys_raw;
    vp.key_info = ctx->d_key_info;
    vp.key_tab = ctx->d_key_tab;
    vp.key_stride = ctx->key_words;
    vp.key_negtab = ctx->key_negtab ? 1u : 0u;
    vp.nkeys = (uint32_t)ctx->nkeys;
    vp.btab = ctx->d_btab;
    static const uint8_t kNoSeed[32] = {0};   // strict-only calls draw no coefficients
    std::memcpy(vp.zseed, zseed ? zseed : kNoSeed, 32);
    vp.flags = d_flags;
    vp.slow_count = slow_count;
    vp.slow_list = ws->w_slow_list.as<uint32_t>();
    vp.slow_slot = ws->w_slow_slot.as<uint32_t>();
    vp.slow_buf = ws->w_slow_buf.as<uint32_t>();
    vp.pslow = batch_mode ? ws->w_pslow.as<uint32_t>() : nullptr;
    vp.cert_state = cert_state;
    vp.ok_out = batch_mode ? nullptr : d_sig_ok;
    vp.pbuf = ws->w_pbuf.as<uint32_t>();
    vp.pre = ws->w_pre.as<uint32_t>();
    vp.perm = nullptr;
    vp.pinfo = nullptr;
    if (group) {
        NW_TRY(launch_group_scatter((uint32_t)nsigs, (uint32_t)ctx->nkeys, d_signer, sig_cert,
                                    ws->w_counts.as<uint32_t>(), ws->w_cursor.as<uint32_t>(), ws->w_perm.as<uint32_t>(),
                                    ws->w_pinfo.as<uint2>(), st),
               "signer grouping");
        vp.perm = ws->w_perm.as<uint32_t>();
        vp.pinfo = ws->w_pinfo.as<uint2>();
    }
    vp.g0 = 0;
    vp.gn = (uint32_t)nsigs;
    vp.fk = finish_k_for(ctx, nsigs);
    hipEvent_t ev_stop = nullptr;
    {
        std::lock_guard<std::mutex> g(ctx->prof_mu);
        if (ctx->prof_on && nsigs) {
            if (ctx->prof_used == ctx->prof_events.size()) {
                hipEvent_t a, b;
                NW_TRY(hipEventCreate(&a), "hipEventCreate");
                NW_TRY(hipEventCreate(&b), "hipEventCreate");
                ctx->prof_events.emplace_back(a, b);
            }
            NW_TRY(hipEventRecord(ctx->prof_events[ctx->prof_used].first, st), "hipEventRecord");
            ev_stop = ctx->prof_events[ctx->prof_used].second;
            ++ctx->prof_used;
            ctx->prof_sigs += nsigs;
        }
    }
    NW_TRY(launch_verify(vp, msgmode, ctx->key_window, st), "k_verify");
    // brackets k_verify alone, or k_verify_split + the finish fused into it (split_fuses_finish:
    // launches of <= 4,096 signatures; nwcrypto.h, nw_profile_read)
    if (ev_stop) NW_TRY(hipEventRecord(ev_stop, st), "hipEventRecord");
    // small launches: k_verify_split has done k_finish's work itself (split_fuses_finish)
    if (!split_fuses_finish(vp.gn, vp.fk)) NW_TRY(launch_finish(vp, st), "k_finish");
    if (!batch_mode) return NW_OK;   // strict verdicts only (bytes written by k_finish): no certificate pass

    FinalizeParams fp{};
    fp.ncerts = (uint32_t)ncerts;
    fp.nsigs = (uint32_t)nsigs;
    fp.cert_first = d_first;
    fp.cert_n = d_nv;
    fp.flags = d_flags;
    fp.signer = d_signer;
    fp.sig_cert = sig_cert;
    fp.stake = ctx->d_stake;
    fp.slow_slot = vp.slow_slot;
    fp.slow_buf = vp.slow_buf;
    fp.cert_state = vp.cert_state;
    fp.cert_ok = d_cert_ok;
    fp.accepted_stake = d_stake_out;
    fp.sig_ok = d_sig_ok;
    fp.exact_count = slow_count + 1;   // word 1 of the zeroed slow-path counter block
    fp.exact_list = ws->w_exact.as<uint32_t>();
    if (slow_tail_fits(ncerts, nsigs)) {   // one header / vote batch: exact path + finalize in one launch
        NW_TRY(launch_slow_tail(vp, fp, msgmode, ctx->key_window, st), "k_slow_tail");
        return NW_OK;
    }
    NW_TRY(launch_slow(vp, msgmode, ctx->key_window, (uint32_t)nsigs, st), "k_slow_prep / k_slow_mul");
    NW_TRY(launch_finalize(fp, st), "k_cert_finalize / k_cert_exact");
    return NW_OK;
}

// Host-buffer inputs of one call: segments are packed into the workspace's pinned buffer (256-B
// aligned) and copied to their device buffers with asynchronous DMAs, so a call issues no
// pageable copies and no intermediate synchronization (the call's final stream sync releases the
// buffer).  Every segment is staged, large ones included: the runtime's pageable H2D runs at the
// pinned rate only for host pages it has already seen; the first copy from a fresh buffer pins its
// pages and took 7-10 ms per 8 MB on MI355X (profiles/r04/host_fed_trace_r04h.txt), and a node's
// input buffers are fresh on every call (network receives).  The staging memcpy costs ~0.3 ms per
// 8 MB at 31-34 GB/s (tools/host_fed_probe.py).
// Calls whose whole input fits this many bytes take the one-DMA small-call path.
constexpr size_t kSmallCallBytes = 2u << 20;

class Stager {
public:
    Stager(Workspace* ws, hipStream_t st) : ws_(ws), st_(st) {}
    // upper bound of the staged bytes of the call (one allocation, before any segment)
    hipError_t reserve(size_t bytes) { return ws_->h_io.ensure(bytes + 16 * 256); }
    static size_t room(size_t bytes) { return align256(bytes); }
    uint8_t* alloc(size_t n) {
        uint8_t* h = ws_->h_io.bytes() + off_;
        off_ = align256(off_ + n);
        return h;
    }
    hipError_t copy(void* dst, const uint8_t* h, size_t n) {
        return n ? hipMemcpyAsync(dst, h, n, hipMemcpyHostToDevice, st_) : hipSuccess;
    }
    hipError_t put(void* dst, const void* src, size_t n);

private:
    Workspace* ws_;
    hipStream_t st_;
    size_t off_ = 0;
};

// Upload n bytes of host memory through pinned staging at h: 4 MiB chunks, each chunk's DMA issued
// as soon as it is staged, so the DMA of one chunk overlaps the memcpy of the next.
constexpr size_t kStageChunk = 4u << 20;

// Large uploads (a window of worker batches is ~640 MB) are staged by several threads: one thread's memcpy into pinned memory runs at ~22 GB/s on the
// box's EPYC host, below the ~55 GB/s PCIe DMA behind it.  Chunk c covers staging bytes
// [cb[c], cb[c+1]); copy_chunk(c) fills it.  Helper threads and the calling thread take chunks from
// a shared counter, and the calling thread issues the DMAs strictly in chunk order, each as soon as
// its chunk is staged, so the uploads still overlap the staging.  Helpers are started per call
// (tens of microseconds against milliseconds of copying), at most kMaxStageHelpers across all
// concurrent calls (host-buffer calls from many threads must not oversubscribe the host); below
// kStageParallelMin bytes everything stays on the calling thread.  (Helpers from 2 MiB up, with
// 1 MiB chunks, left the uncached-key call unchanged (50.2 M sigs/s) and measured the worker
// digest windows slower on the same run, r04v.)
constexpr size_t kStageParallelMin = 32u << 20;
constexpr unsigned kStageThreads = 8;           // per call, including the calling thread
constexpr int kMaxStageHelpers = 8;             // across calls; the box's cgroup quota is 16 CPUs
std::atomic<int> g_stage_helpers{0};

template <class CopyChunk>
hipError_t stage_chunks(size_t nch, const size_t* cb, CopyChunk&& copy_chunk, const uint8_t* h, uint8_t* d,
                        hipStream_t st) {
    auto dma = [&](size_t c) {
        return hipMemcpyAsync(d + cb[c], h + cb[c], cb[c + 1] - cb[c], hipMemcpyHostToDevice, st);
    };
    size_t want = cb[nch] - cb[0] >= kStageParallelMin ? std::min<size_t>(kStageThreads - 1, nch / 2) : 0;
    size_t helpers = 0;
    while (helpers < want) {   // reserve helper slots from the process-wide cap
        int cur = g_stage_helpers.load(std::memory_order_relaxed);
        if (cur >= kMaxStageHelpers) break;
        if (g_stage_helpers.compare_exchange_weak(cur, cur + 1, std::memory_order_relaxed)) ++helpers;
    }
    struct Release {
        size_t n;
        ~Release() { if (n) g_stage_helpers.fetch_sub((int)n, std::memory_order_relaxed); }
    } release{helpers};
    if (helpers == 0) {
        for (size_t c = 0; c < nch; ++c) {
            copy_chunk(c);
            const hipError_t e = dma(c);
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
    std::atomic<size_t> next{0};
    std::unique_ptr<std::atomic<uint8_t>[]> ready(new std::atomic<uint8_t>[nch]);
    for (size_t c = 0; c < nch; ++c) ready[c].store(0, std::memory_order_relaxed);
    auto take = [&]() {
        const size_t c = next.fetch_add(1, std::memory_order_relaxed);
        if (c >= nch) return false;
        copy_chunk(c);
        ready[c].store(1, std::memory_order_release);
        return true;
    };
    std::vector<std::thread> pool;
    pool.reserve(helpers);
    for (size_t t = 0; t < helpers; ++t) {
        try {
            pool.emplace_back([&] { while (take()) {} });
        } catch (const std::system_error&) {
            break;   // fewer helpers (the calling thread copies whatever is left)
        }
    }
    hipError_t err = hipSuccess;
    for (size_t sent = 0; sent < nch;) {
        if (ready[sent].load(std::memory_order_acquire)) {
            if (err == hipSuccess) err = dma(sent);
            ++sent;
        } else if (!take()) {
            std::this_thread::yield();
        }
    }
    for (auto& t : pool) t.join();
    return err;
}

hipError_t staged_h2d(uint8_t* h, uint8_t* dst, const uint8_t* src, size_t n, hipStream_t st) {
    if (n == 0) return hipSuccess;
    const size_t nch = (n + kStageChunk - 1) / kStageChunk;
    std::vector<size_t> cb(nch + 1);
    for (size_t c = 0; c < nch; ++c) cb[c] = c * kStageChunk;
    cb[nch] = n;
    return stage_chunks(nch, cb.data(), [&](size_t c) { std::memcpy(h + cb[c], src + cb[c], cb[c + 1] - cb[c]); },
                        h, dst, st);
}

// Mid-size uploads (an uncached-key call's 4 MB of signatures) go in kPutPiece pieces, each DMA
// issued once its piece is staged, so the memcpy of one piece runs under the DMA of the previous.
constexpr size_t kPutPiece = 1u << 20;

hipError_t Stager::put(void* dst, const void* src, size_t n) {
    if (!n) return hipSuccess;
    uint8_t* h = alloc(n);
    if (n >= kStageParallelMin) return staged_h2d(h, static_cast<uint8_t*>(dst), static_cast<const uint8_t*>(src), n, st_);
    const size_t piece = n >= 2 * kPutPiece ? kPutPiece : n;
    for (size_t o = 0; o < n; o += piece) {
        const size_t m = std::min(piece, n - o);
        std::memcpy(h + o, static_cast<const uint8_t*>(src) + o, m);
        const hipError_t e = copy(static_cast<uint8_t*>(dst) + o, h + o, m);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

size_t message_bytes(const size_t* len, size_t n) {
    size_t total = 0;
    for (size_t i = 0; i < n; ++i) total += len[i];
    return total;
}

// Staged bytes of upload_messages (the packed messages, offsets and lengths).
size_t message_stage_bytes(size_t total, size_t n) { return align256(total + 8) + 2 * align256(n * 8 + 8); }

// Pack per-signature messages into the workspace (MSGMODE 1).
int upload_messages(nw_ctx* ctx, Workspace* ws, Stager& sg, const uint8_t* const* msg, const size_t* len, size_t n,
                    size_t total, uint64_t* fixed_len = nullptr) {
    NW_TRY(ws->ensure(ws->w_msg, total + 8), "ws msg");
    if (fixed_len) {
        // messages of one length laid out back to back (the worker's 8-byte messages, numpy rows):
        // one block, no offset / length arrays (*fixed_len = the length; UINT64_MAX otherwise)
        bool ok = n > 0;
        for (size_t i = 1; ok && i < n; ++i) ok = len[i] == len[0] && msg[i] == msg[0] + i * len[0];
        *fixed_len = ok ? (uint64_t)len[0] : UINT64_MAX;
        if (ok) {
            uint8_t* packed = sg.alloc(total + 8);
            if (total) std::memcpy(packed, msg[0], total);
            std::memset(packed + total, 0, 8);
            NW_TRY(sg.copy(ws->w_msg.p, packed, total + 8), "H2D msg");
            return NW_OK;
        }
    }
    NW_TRY(ws->ensure(ws->w_msg_off, n * 8 + 8), "ws msg_off");
    NW_TRY(ws->ensure(ws->w_msg_len, n * 8 + 8), "ws msg_len");
    uint8_t* packed = sg.alloc(total + 8);
    uint64_t* off = reinterpret_cast<uint64_t*>(sg.alloc(n * 8 + 8));
    uint64_t* ln = reinterpret_cast<uint64_t*>(sg.alloc(n * 8 + 8));
    // messages laid out back to back in the caller's memory (the worker's fixed 8-byte messages,
    // numpy rows) are copied as one block instead of one memcpy each
    bool contiguous = n > 0;
    size_t pos = 0;
    for (size_t i = 0; i < n; ++i) {
        off[i] = pos;
        ln[i] = len[i];
        contiguous = contiguous && msg[i] == msg[0] + pos;
        pos += len[i];
    }
    if (contiguous) {
        if (pos) std::memcpy(packed, msg[0], pos);
    } else {
        for (size_t i = 0; i < n; ++i)
            if (len[i]) std::memcpy(packed + off[i], msg[i], len[i]);
    }
    std::memset(packed + pos, 0, 8);
    NW_TRY(sg.copy(ws->w_msg.p, packed, total + 8), "H2D msg");
    NW_TRY(sg.copy(ws->w_msg_off.p, reinterpret_cast<uint8_t*>(off), n * 8), "H2D off");
    NW_TRY(sg.copy(ws->w_msg_len.p, reinterpret_cast<uint8_t*>(ln), n * 8), "H2D len");
    return NW_OK;
}

// Strict verify of signatures whose keys are not cached: k_verify_var + k_finish (messages, sigs
// and raw keys already uploaded to the workspace).
int enqueue_strict_var(nw_ctx* ctx, Workspace* ws, size_t n, hipStream_t st, uint8_t* d_ok = nullptr) {
    NW_TRY(ws->ensure(ws->w_flags, n * 4 + 4), "ws flags");
    NW_TRY(ws->ensure(ws->w_sig_cert, n * 4 + 4), "ws sig_cert");
    NW_TRY(ws->ensure(ws->w_pbuf, n * (size_t)PBUF_WORDS * 4 + 16), "ws pbuf");
    NW_TRY(ws->ensure(ws->w_pre, n * 40 + 16), "ws pre");
    NW_TRY(ws->ensure(ws->w_var, n * 320 * 4 + 16), "ws var table");
    NW_TRY(hipMemsetAsync(ws->w_sig_cert.p, 0, n * 4 + 4, st), "memset sig_cert");
    VerifyParams vp{};
    vp.n = (uint32_t)n;
    vp.g0 = 0;
    vp.gn = (uint32_t)n;
    vp.fk = finish_k_for(ctx, n);
    vp.batch_mode = 0;
    vp.sig = ws->w_sig.as<uint8_t>();
    vp.sig_keys = ws->w_keys.as<uint32_t>();
    vp.sig_cert = ws->w_sig_cert.as<uint32_t>();
    vp.msg_base = ws->w_msg.as<uint8_t>();
    vp.msg_off = ws->w_msg_off.as<uint64_t>();
    vp.msg_len = ws->w_msg_len.as<uint64_t>();
    vp.btab = ctx->d_btab;
    vp.flags = ws->w_flags.as<uint32_t>();
    vp.pbuf = ws->w_pbuf.as<uint32_t>();
    vp.pre = ws->w_pre.as<uint32_t>();
    vp.ok_out = d_ok;   // verdict bytes straight from k_finish
    NW_TRY(launch_verify_var(vp, 1, ws->w_var.as<uint32_t>(), st), "k_verify_var");
    NW_TRY(launch_finish(vp, st), "k_finish");
    return NW_OK;
}

// Randomized batch verify of nb consecutive batches (batch b = the next counts[b] signatures)
// without the key cache: the Pippenger MSM of nw_msm.hip.  Messages, sigs and raw keys are in the
// workspace.  Writes batch_ok (device, may be null) and/or point_out (device, [nb][40], may be null);
// bad_out (device, [nb] u32) receives the parse/decode failure flags.
int enqueue_msm(nw_ctx* ctx, Workspace* ws, size_t nb, const uint32_t* counts, size_t nsig, const uint8_t* zseed,
                uint64_t batch_base, uint32_t z_off, uint8_t* d_batch_ok, uint32_t* d_point_out, uint32_t** d_bad_out,
                hipStream_t st, uint64_t msg_flen) {
    uint32_t nmax = 0;
    for (size_t b = 0; b < nb; ++b) nmax = counts[b] > nmax ? counts[b] : nmax;
    const uint32_t C = nmax >= 512 ? 8 : 7;
    const uint32_t NA = (uint32_t)msm_nwin_a((int)C), NR = (uint32_t)msm_nwin_r((int)C);
    const uint32_t B = 1u << (C - 1);
    std::vector<uint32_t> bfirst(nb), bcount(nb), sig_batch(nsig), wfirst(nb * NA + 1);
    std::vector<MsmTask> tasks;
    size_t f = 0;
    for (size_t b = 0; b < nb; ++b) {
        bfirst[b] = (uint32_t)f;
        bcount[b] = counts[b];
        for (uint32_t t = 0; t < counts[b]; ++t) sig_batch[f + t] = (uint32_t)b;
        for (uint32_t j = 0; j < NA; ++j) {
            wfirst[b * NA + j] = (uint32_t)tasks.size();
            const size_t lo = 2 * f + (j < NR ? 0 : counts[b]), hi = 2 * f + 2 * (size_t)counts[b];
            for (size_t e = lo; e < hi; e += MSM_CH) {
                const size_t e1 = e + MSM_CH < hi ? e + MSM_CH : hi;
                tasks.push_back(MsmTask{(uint32_t)e, (uint32_t)e1, j, (uint32_t)tasks.size()});
            }
        }
        f += counts[b];
    }
    wfirst[nb * NA] = (uint32_t)tasks.size();
    const size_t ntasks = tasks.size();
    // metadata block: bfirst | bcount | sig_batch | wfirst | tasks | bad | batch verdict scratch
    const size_t o_bfirst = 0, o_bcount = align256(nb * 4), o_sb = o_bcount + align256(nb * 4),
                 o_wf = o_sb + align256(nsig * 4 + 4), o_tasks = o_wf + align256(wfirst.size() * 4),
                 o_bad = o_tasks + align256(ntasks * sizeof(MsmTask) + 16), meta = o_bad + align256(nb * 4);
    NW_TRY(ws->ensure(ws->w_msm_meta, meta), "ws msm meta");
    NW_TRY(ws->ensure(ws->w_msm_ent, 2 * nsig * MSM_ENT_WORDS * 4 + 16), "ws msm entries");
    NW_TRY(ws->ensure(ws->w_msm_dig, (size_t)NA * 2 * nsig * 2 + 16), "ws msm digits");
    NW_TRY(ws->ensure(ws->w_msm_zs, (size_t)MSM_ZS_WORDS * nsig * 4 + 16), "ws msm zs");
    NW_TRY(ws->ensure(ws->w_msm_bkt, ntasks * B * MSM_PT_WORDS * 4 + 16), "ws msm buckets");
    NW_TRY(ws->ensure(ws->w_msm_part, ntasks * 128 * MSM_PT_WORDS * 4 + 16), "ws msm partials");
    NW_TRY(ws->ensure(ws->w_msm_wpart, (ntasks + nb * NA) * MSM_PT_WORDS * 4 + 16), "ws msm window sums");
    // staged in the workspace's second pinned buffer (every caller synchronizes before returning)
    NW_TRY(ws->h_meta.ensure(meta), "pinned msm meta");
    uint8_t* hmeta = ws->h_meta.bytes();
    std::memset(hmeta, 0, meta);
    std::memcpy(hmeta + o_bfirst, bfirst.data(), nb * 4);
    std::memcpy(hmeta + o_bcount, bcount.data(), nb * 4);
    if (nsig) std::memcpy(hmeta + o_sb, sig_batch.data(), nsig * 4);
    std::memcpy(hmeta + o_wf, wfirst.data(), wfirst.size() * 4);
    if (ntasks) std::memcpy(hmeta + o_tasks, tasks.data(), ntasks * sizeof(MsmTask));
    uint8_t* dm = ws->w_msm_meta.as<uint8_t>();
    NW_TRY(hipMemcpyAsync(dm, hmeta, meta, hipMemcpyHostToDevice, st), "H2D msm meta");
    MsmParams mp{};
    mp.nb = (uint32_t)nb;
    mp.nsig = (uint32_t)nsig;
    mp.c = C;
    mp.bfirst = reinterpret_cast<const uint32_t*>(dm + o_bfirst);
    mp.bcount = reinterpret_cast<const uint32_t*>(dm + o_bcount);
    mp.sig_batch = reinterpret_cast<const uint32_t*>(dm + o_sb);
    mp.sig = ws->w_sig.as<uint8_t>();
    mp.keys = ws->w_keys.as<uint32_t>();
    mp.msg_base = ws->w_msg.as<uint8_t>();
    mp.msg_off = ws->w_msg_off.as<uint64_t>();
    mp.msg_len = ws->w_msg_len.as<uint64_t>();
    mp.msg_flen = msg_flen;
    mp.batch_base = batch_base;
    mp.z_off = z_off;
    std::memcpy(mp.zseed, zseed, 32);
    mp.ent = ws->w_msm_ent.as<uint32_t>();
    mp.dig = ws->w_msm_dig.as<int16_t>();
    mp.zs = ws->w_msm_zs.as<uint32_t>();
    mp.bad = reinterpret_cast<uint32_t*>(dm + o_bad);
    mp.tasks = reinterpret_cast<const MsmTask*>(dm + o_tasks);
    mp.ntasks = (uint32_t)ntasks;
    mp.bkt = ws->w_msm_bkt.as<uint32_t>();
    mp.part = ws->w_msm_part.as<uint32_t>();
    mp.wpart = ws->w_msm_wpart.as<uint32_t>();
    mp.wfirst = reinterpret_cast<const uint32_t*>(dm + o_wf);
    mp.one_task_windows = 1;
    for (size_t k = 0; k < nb * NA; ++k)
        if (wfirst[k + 1] - wfirst[k] != 1u || wfirst[k] != k) mp.one_task_windows = 0;
    mp.btab = ctx->d_btab;
    mp.batch_ok = d_batch_ok;
    mp.point_out = d_point_out;
    NW_TRY(launch_msm(mp, st), "k_msm");
    if (d_bad_out) *d_bad_out = mp.bad;
    return NW_OK;
}

// Upload per-signature messages, signatures and raw keys to the workspace (uncached-key paths).
// fixed_len (MSM callers, whose kernel reads either form): see upload_messages.
int upload_sig_keys(nw_ctx* ctx, Workspace* ws, const uint8_t* const* msg, const size_t* len,
                    const uint8_t (*pk)[32], const uint8_t (*sig)[64], size_t n, hipStream_t st,
                    uint64_t* fixed_len = nullptr) {
    const size_t total = message_bytes(len, n);
    Stager sg(ws, st);
    NW_TRY(sg.reserve(message_stage_bytes(total, n) + Stager::room(n * 64) + Stager::room(n * 32)), "pinned io");
    int rc = upload_messages(ctx, ws, sg, msg, len, n, total, fixed_len);
    if (rc != NW_OK) return rc;
    NW_TRY(ws->ensure(ws->w_sig, n * 64 + 64), "ws sig");
    NW_TRY(ws->ensure(ws->w_keys, n * 32 + 32), "ws keys");
    NW_TRY(sg.put(ws->w_sig.p, sig, n * 64), "H2D sig");
    NW_TRY(sg.put(ws->w_keys.p, pk, n * 32), "H2D keys");
    return NW_OK;
}

// Staged bytes of run_generic's one-DMA layout (messages, offsets, lengths, sigs, slots, the
// certificate word pair and the preamble state).
size_t packed_bytes(size_t total, size_t n) {
    return align256(total + 8) + 2 * align256(n * 8) + align256(n * 64) + align256(n * 4) + 256 +
           prestaged_bytes(n, 1);
}

// Shared body of strict_many / verify_batch: every signature in one "certificate" 0.  Cached keys
// take the comb path; a call with any key outside the cache takes the variable-base path (strict:
// k_verify_var; batch: the MSM) and leaves the cache unchanged.
int run_generic(nw_ctx* ctx, const uint8_t* const* msg, const size_t* len, const uint8_t (*pk)[32],
                const uint8_t (*sig)[64], size_t n, const uint8_t* zseed, uint64_t batch_index, uint32_t batch_mode,
                uint8_t* ok_out, uint8_t* verdict_out) {
    std::shared_lock<std::shared_mutex> keys(ctx->keys_mu);
    Lease lease(ctx);
    Workspace* ws = lease.ws();
    if (!ws) {
        set_error(ctx, "workspace allocation failed");
        return NW_ERR_DEVICE;
    }
    hipStream_t st = ws->stream;
    NW_TRY(lease.bind(st, true), "hipStreamWaitEvent");
    std::vector<uint32_t> slots(n);
    const bool cached = lookup_slots(ctx, pk, n, slots.data());
    int rc = NW_OK;
    if (!cached) {
        uint64_t flen = UINT64_MAX;
        rc = upload_sig_keys(ctx, ws, msg, len, pk, sig, n, st, batch_mode ? &flen : nullptr);
        if (rc != NW_OK) return rc;
        NW_TRY(ws->ensure(ws->w_ok, n + 16), "ws ok");
        if (batch_mode) {
            NW_TRY(ws->ensure(ws->w_cert_ok, 16), "ws verdict");
            const uint32_t cnt = (uint32_t)n;
            rc = enqueue_msm(ctx, ws, 1, &cnt, n, zseed, batch_index, 0, ws->w_cert_ok.as<uint8_t>(), nullptr, nullptr,
                             st, flen);
            if (rc != NW_OK) return rc;
        } else {
            rc = enqueue_strict_var(ctx, ws, n, st, ws->w_ok.as<uint8_t>());
            if (rc != NW_OK) return rc;
        }
    } else if (n <= kStagedMaxSigs && packed_bytes(message_bytes(len, n), n) < kSmallCallBytes) {
        // one-message paths (Signature::verify, one certificate's verify_batch): every input and the
        // preamble state in ONE staged H2D, no preamble kernels, both outputs in ONE D2H
        const size_t total = message_bytes(len, n);
        const size_t o_msg = 0, o_off = align256(total + 8), o_len = o_off + align256(n * 8),
                     o_sig = o_len + align256(n * 8), o_signer = o_sig + align256(n * 64),
                     o_fn = o_signer + align256(n * 4), o_pre = o_fn + 256,
                     in_bytes = o_pre + prestaged_bytes(n, 1);
        const size_t o_cok = 0, o_ok = 256, out_bytes = align256(256 + n);
        NW_TRY(ws->ensure(ws->w_io, in_bytes + out_bytes), "ws io");
        NW_TRY(ws->h_io.ensure(in_bytes > out_bytes ? in_bytes : out_bytes), "pinned io");
        uint8_t* h = ws->h_io.bytes();
        uint8_t* d = ws->w_io.as<uint8_t>();
        uint8_t* d_out = d + in_bytes;
        uint64_t* hoff = reinterpret_cast<uint64_t*>(h + o_off);
        uint64_t* hlen = reinterpret_cast<uint64_t*>(h + o_len);
        size_t pos = 0;
        for (size_t i = 0; i < n; ++i) {
            hoff[i] = pos;
            hlen[i] = len[i];
            if (len[i]) std::memcpy(h + o_msg + pos, msg[i], len[i]);
            pos += len[i];
        }
        std::memset(h + o_msg + pos, 0, 8);
        std::memcpy(h + o_sig, sig, n * 64);
        std::memcpy(h + o_signer, slots.data(), n * 4);
        uint32_t* fn = reinterpret_cast<uint32_t*>(h + o_fn);
        fn[0] = 0;
        fn[1] = (uint32_t)n;
        PreStaged pre{};
        prestage(h + o_pre, d + o_pre, fn, fn + 1, 1, n, pre);
        NW_TRY(hipMemcpyAsync(d, h, in_bytes, hipMemcpyHostToDevice, st), "H2D inputs");
        rc = enqueue_certs(ctx, ws, 1, reinterpret_cast<const uint32_t*>(d + o_fn),
                           reinterpret_cast<const uint32_t*>(d + o_fn + 4), n, d + o_sig,
                           reinterpret_cast<const uint32_t*>(d + o_signer), 1, nullptr, d + o_msg,
                           reinterpret_cast<const uint64_t*>(d + o_off), reinterpret_cast<const uint64_t*>(d + o_len),
                           zseed, batch_index, batch_mode, d_out + o_cok, nullptr, nullptr, st,
                           ok_out ? d_out + o_ok : nullptr, nullptr, &pre);
        if (rc != NW_OK) return rc;
        // the H2D above has completed in stream order before this copy overwrites the staging buffer
        NW_TRY(hipMemcpyAsync(h, d_out, out_bytes, hipMemcpyDeviceToHost, st), "D2H outputs");
        NW_TRY(hipStreamSynchronize(st), "sync");
        lease.synced();
        if (ok_out) std::memcpy(ok_out, h + o_ok, n);
        if (verdict_out) *verdict_out = h[o_cok];
        return NW_OK;
    } else {
        const size_t total = message_bytes(len, n);
        Stager sg(ws, st);
        NW_TRY(sg.reserve(message_stage_bytes(total, n) + Stager::room(n * 64) + Stager::room(n * 4) + 512),
               "pinned io");
        rc = upload_messages(ctx, ws, sg, msg, len, n, total);
        if (rc != NW_OK) return rc;
        NW_TRY(ws->ensure(ws->w_sig, n * 64), "ws sig");
        NW_TRY(ws->ensure(ws->w_signer, n * 4), "ws signer");
        NW_TRY(ws->ensure(ws->w_cert_first, 16), "ws first");
        NW_TRY(ws->ensure(ws->w_cert_n, 16), "ws n");
        NW_TRY(ws->ensure(ws->w_cert_ok, 16), "ws cert_ok");
        NW_TRY(ws->ensure(ws->w_ok, n + 16), "ws ok");
        const uint32_t first = 0, nv = (uint32_t)n;
        NW_TRY(sg.put(ws->w_sig.p, sig, n * 64), "H2D sig");
        NW_TRY(sg.put(ws->w_signer.p, slots.data(), n * 4), "H2D signer");
        NW_TRY(sg.put(ws->w_cert_first.p, &first, 4), "H2D first");
        NW_TRY(sg.put(ws->w_cert_n.p, &nv, 4), "H2D n");
        rc = enqueue_certs(ctx, ws, 1, ws->w_cert_first.as<uint32_t>(), ws->w_cert_n.as<uint32_t>(), n,
                           ws->w_sig.as<uint8_t>(), ws->w_signer.as<uint32_t>(), 1, nullptr, ws->w_msg.as<uint8_t>(),
                           ws->w_msg_off.as<uint64_t>(), ws->w_msg_len.as<uint64_t>(), zseed, batch_index, batch_mode,
                           ws->w_cert_ok.as<uint8_t>(), nullptr, nullptr, st,
                           ok_out ? ws->w_ok.as<uint8_t>() : nullptr);   // verdict bytes from k_cert_finalize
        if (rc != NW_OK) return rc;
    }
    if (ok_out) NW_TRY(hipMemcpyAsync(ok_out, ws->w_ok.p, n, hipMemcpyDeviceToHost, st), "D2H ok");
    if (verdict_out) NW_TRY(hipMemcpyAsync(verdict_out, ws->w_cert_ok.p, 1, hipMemcpyDeviceToHost, st), "D2H");
    NW_TRY(hipStreamSynchronize(st), "sync");
    lease.synced();
    return NW_OK;
}

bool zseed_ok(nw_ctx* ctx, const uint8_t* zseed) {
    if (zseed) return true;
    set_error(ctx, "zseed is NULL: batch coefficients need a fresh 32-byte CSPRNG seed per call");
    return false;
}

}  // namespace

extern "C" {

const char* nw_version(void) { return "nwcrypto 0.4 gfx950 src " NW_SRC_HASH " commit " NW_SRC_COMMIT; }

int nw_abi_version(void) { return NW_ABI_VERSION; }

namespace {
// The basepoint comb (one "key" = B; with its negated copy when B_NEGTAB) is shared by every context
// of the process on a device, reference-counted: a node running its primary's and its workers'
// engines in one process holds one copy (11.8 GB per table at W24, 42.9 GB at W26).  The registry is
// never destroyed (contexts may be released during interpreter shutdown).
struct BaseTable {
    uint32_t* p = nullptr;
    int refs = 0;
};
std::mutex& base_mu() {
    static std::mutex* m = new std::mutex();
    return *m;
}
std::unordered_map<int, BaseTable>& base_tables() {
    static auto* t = new std::unordered_map<int, BaseTable>();
    return *t;
}

int acquire_base(nw_ctx* ctx) {
    std::lock_guard<std::mutex> g(base_mu());
    BaseTable& b = base_tables()[ctx->device];
    if (!b.p) {
        uint32_t* tab = nullptr;
        uint32_t* d_braw = nullptr;
        uint32_t* d_binfo = nullptr;
        int rc = NW_OK;
        if (hipMalloc(&tab, B_TABLES * comb_words(B_WINDOW) * 4) != hipSuccess || hipMalloc(&d_braw, 32) != hipSuccess ||
            hipMalloc(&d_binfo, 16) != hipSuccess)
            rc = NW_ERR_NOMEM;
        if (rc == NW_OK && hipMemcpy(d_braw, kBaseEnc, 32, hipMemcpyHostToDevice) != hipSuccess) rc = NW_ERR_DEVICE;
        if (rc == NW_OK)
            rc = build_keys(ctx, d_braw, d_binfo, tab, 1, B_WINDOW, B_TABLES * comb_words(B_WINDOW), B_NEGTAB);
        if (hipStreamSynchronize(ctx->stream) != hipSuccess && rc == NW_OK) rc = NW_ERR_DEVICE;
        ctx->w_bases.release();   // the basepoint's bases scratch is not the committee's
        for (uint32_t* q : {d_braw, d_binfo})
            if (q) (void)hipFree(q);
        if (rc != NW_OK) {
            if (tab) (void)hipFree(tab);
            return rc;
        }
        b.p = tab;
    }
    ++b.refs;
    ctx->d_btab = b.p;
    return NW_OK;
}

void release_base(nw_ctx* ctx) {
    if (!ctx->d_btab) return;
    std::lock_guard<std::mutex> g(base_mu());
    BaseTable& b = base_tables()[ctx->device];
    if (--b.refs == 0) {
        (void)hipDeviceSynchronize();   // no other context's work may still read it (none holds it)
        (void)hipFree(b.p);
        b.p = nullptr;
    }
    ctx->d_btab = nullptr;
}
}  // namespace

int nw_ctx_create(nw_ctx** out, const nw_opts* opts) {
    if (!out) return NW_ERR_ARG;
    *out = nullptr;
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev == 0) return NW_ERR_DEVICE;
    int dev = opts && opts->device >= 0 ? opts->device : -1;
    if (dev < 0 && hipGetDevice(&dev) != hipSuccess) return NW_ERR_DEVICE;
    if (dev >= ndev) return NW_ERR_ARG;
    if (opts && (opts->flags & ~NW_OPT_NO_KEY_NEGTAB)) return NW_ERR_ARG;
    if (opts && opts->key_window && opts->key_window != -1 && opts->key_window != 8 && opts->key_window != 9 &&
        opts->key_window != 12 && opts->key_window != 13 && opts->key_window != 16 && opts->key_window != 20)
        return NW_ERR_ARG;
    nw_ctx* ctx = new nw_ctx();
    ctx->device = dev;
    ctx->finish_k = NW_FK_FIXED;
    if (opts) ctx->opt_flags = opts->flags;
    if (opts && opts->max_keys) {
        ctx->max_keys = opts->max_keys;
        ctx->max_keys_user = true;
    }
    if (opts && opts->key_window) {
        ctx->key_window = opts->key_window;
        ctx->committee_mode = ctx->key_window == -1;
    }
    if (hipSetDevice(dev) != hipSuccess || hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
        delete ctx;
        return NW_ERR_DEVICE;
    }
    const int rc = acquire_base(ctx);
    if (rc != NW_OK) {
        nw_ctx_destroy(ctx);
        return rc;
    }
    *out = ctx;
    return NW_OK;
}

void nw_ctx_destroy(nw_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    for (auto& w : ctx->pool) {
        if (w->pending) (void)hipEventSynchronize(w->done);
        if (w->stream) (void)hipStreamSynchronize(w->stream);
        w->release_all();
        if (w->done) (void)hipEventDestroy(w->done);
        if (w->stream) (void)hipStreamDestroy(w->stream);
    }
    ctx->w_bases.release();
    for (auto& ev : ctx->prof_events) {
        (void)hipEventDestroy(ev.first);
        (void)hipEventDestroy(ev.second);
    }
    for (uint32_t* p : {ctx->d_keys_raw, ctx->d_key_info, ctx->d_stake, ctx->d_key_tab})
        if (p) (void)hipFree(p);
    release_base(ctx);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

int nw_profile_enable(nw_ctx* ctx, int on) {
    if (!ctx) return NW_ERR_ARG;
    std::lock_guard<std::mutex> g(ctx->prof_mu);
    ctx->prof_on = on != 0;
    return NW_OK;
}

int nw_profile_read(nw_ctx* ctx, double* verify_ms_total, uint64_t* verify_launches) {
    return nw_profile_read_sigs(ctx, verify_ms_total, verify_launches, nullptr);
}

int nw_profile_read_sigs(nw_ctx* ctx, double* verify_ms_total, uint64_t* verify_launches, uint64_t* verify_sigs) {
    if (!ctx) return NW_ERR_ARG;
    NW_TRY(hipSetDevice(ctx->device), "hipSetDevice");
    std::lock_guard<std::mutex> g(ctx->prof_mu);
    double total = 0;
    for (size_t i = 0; i < ctx->prof_used; ++i) {
        NW_TRY(hipEventSynchronize(ctx->prof_events[i].second), "hipEventSynchronize");
        float ms = 0;
        NW_TRY(hipEventElapsedTime(&ms, ctx->prof_events[i].first, ctx->prof_events[i].second), "elapsed");
        total += ms;
    }
    if (verify_ms_total) *verify_ms_total = total;
    if (verify_launches) *verify_launches = ctx->prof_used;
    if (verify_sigs) *verify_sigs = ctx->prof_sigs;
    ctx->prof_used = 0;
    ctx->prof_sigs = 0;
    return NW_OK;
}

const char* nw_last_error(const nw_ctx* ctx) {
    (void)ctx;
    return tl_last_error.c_str();
}

size_t nw_committee_size(const nw_ctx* ctx) {
    if (!ctx) return 0;
    std::shared_lock<std::shared_mutex> g(const_cast<nw_ctx*>(ctx)->keys_mu);
    return ctx->nkeys;
}

int nw_key_window(const nw_ctx* ctx) {
    if (!ctx) return 0;
    std::shared_lock<std::shared_mutex> g(const_cast<nw_ctx*>(ctx)->keys_mu);
    return ctx->key_window;
}

int nw_key_negtab(const nw_ctx* ctx) {
    if (!ctx) return 0;
    std::shared_lock<std::shared_mutex> g(const_cast<nw_ctx*>(ctx)->keys_mu);
    return ctx->key_negtab ? 1 : 0;
}

int nw_base_window(void) { return B_WINDOW; }

int nw_committee_load(nw_ctx* ctx, const uint8_t (*pk)[32], const uint32_t* stake, size_t n, uint32_t* slot_out) {
    if (!ctx || (!pk && n)) return NW_ERR_ARG;
    NW_TRY(hipSetDevice(ctx->device), "hipSetDevice");
    std::unique_lock<std::shared_mutex> g(ctx->keys_mu);
    std::vector<uint32_t> slots(n);
    int rc = ensure_slots(ctx, pk, stake, n, slots.data());
    if (rc == NW_OK && slot_out && n) std::memcpy(slot_out, slots.data(), n * 4);
    return rc;
}

int nw_verify_strict_many(nw_ctx* ctx, const uint8_t* const* msg, const size_t* len, const uint8_t (*pk)[32],
                          const uint8_t (*sig)[64], size_t n, uint8_t* ok) {
    if (!ctx || !ok || (n && (!msg || !len || !pk || !sig))) return NW_ERR_ARG;
    if (n == 0) return NW_OK;
    if (n > 0xFFFFFFF0u) return NW_ERR_ARG;
    NW_TRY(hipSetDevice(ctx->device), "hipSetDevice");
    return run_generic(ctx, msg, len, pk, sig, n, nullptr, 0, 0, ok, nullptr);
}

int nw_verify_strict(nw_ctx* ctx, const uint8_t* msg, size_t len, const uint8_t pk[32], const uint8_t sig[64]) {
    if (!ctx || !pk || !sig || (len && !msg)) return NW_ERR_ARG;
    uint8_t ok = 0;
    const uint8_t* m = msg ? msg : reinterpret_cast<const uint8_t*>("");
    int rc = nw_verify_strict_many(ctx, &m, &len, reinterpret_cast<const uint8_t(*)[32]>(pk),
                                   reinterpret_cast<const uint8_t(*)[64]>(sig), 1, &ok);
    if (rc != NW_OK) return rc;
    return ok ? NW_OK : NW_ERR_SIG;
}

int nw_verify_batch(nw_ctx* ctx, const uint8_t* const* msg, const size_t* len, const uint8_t (*pk)[32],
                    const uint8_t (*sig)[64], size_t n, const uint8_t zseed[32], uint64_t batch_index) {
    if (!ctx || (n && (!msg || !len || !pk || !sig))) return NW_ERR_ARG;
    if (!zseed_ok(ctx, zseed)) return NW_ERR_ARG;
    if (n == 0) return NW_OK;   // empty batch: the MSM is (-0)B = identity -> Ok
    if (n > 0xFFFFFFF0u) return NW_ERR_ARG;
    NW_TRY(hipSetDevice(ctx->device), "hipSetDevice");
    uint8_t verdict = 0;
    int rc = run_generic(ctx, msg, len, pk, sig, n, zseed, batch_index, 1, nullptr, &verdict);
    if (rc != NW_OK) return rc;
    return verdict ? NW_OK : NW_ERR_SIG;
}

int nw_verify_batches_pk(nw_ctx* ctx, size_t nb, const uint32_t* counts, const uint8_t* const* msg,
                         const size_t* len, const uint8_t (*pk)[32], const uint8_t (*sig)[64],
                         const uint8_t zseed[32], uint64_t batch_base, uint8_t* batch_ok) {
    if (!ctx || (nb && (!counts || !batch_ok))) return NW_ERR_ARG;
    if (!zseed_ok(ctx, zseed)) return NW_ERR_ARG;
    size_t nsig = 0;
    for (size_t b = 0; b < nb; ++b) nsig += counts[b];
    if (nsig && (!msg || !len || !pk || !sig)) return NW_ERR_ARG;
    if (nsig > 0x7FFFFFF0u) return NW_ERR_ARG;
    if (nb == 0) return NW_OK;
    NW_TRY(hipSetDevice(ctx->device), "hipSetDevice");
    std::shared_lock<std::shared_mutex> keys(ctx->keys_mu);
    Lease lease(ctx);
    Workspace* ws = lease.ws();
    if (!ws) return NW_ERR_DEVICE;
    hipStream_t st = ws->stream;
    NW_TRY(lease.bind(st, true), "hipStreamWaitEvent");
    uint64_t flen = UINT64_MAX;
    int rc = upload_sig_keys(ctx, ws, msg, len, pk, sig, nsig, st, &flen);
    if (rc != NW_OK) return rc;
    NW_TRY(ws->ensure(ws->w_cert_ok, nb + 16), "ws verdicts");
    rc = enqueue_msm(ctx, ws, nb, counts, nsig, zseed, batch_base, 0, ws->w_cert_ok.as<uint8_t>(), nullptr, nullptr,
                     st, flen);
    if (rc != NW_OK) return rc;
    NW_TRY(hipMemcpyAsync(batch_ok, ws->w_cert_ok.p, nb, hipMemcpyDeviceToHost, st), "D2H verdicts");
    NW_TRY(hipStreamSynchronize(st), "sync");
    lease.synced();
    return NW_OK;
}

int nw_verify_batch_partial(nw_ctx* ctx, const uint8_t* const* msg, const size_t* len, const uint8_t (*pk)[32],
                            const uint8_t (*sig)[64], size_t n, const uint8_t zseed[32], uint64_t batch_index,
                            uint32_t z_offset, uint8_t point[NW_POINT_BYTES], int* bad) {
    if (!ctx || !point || !bad || (n && (!msg || !len || !pk || !sig))) return NW_ERR_ARG;
    if (!zseed_ok(ctx, zseed)) return NW_ERR_ARG;
    if (n > 0x7FFFFFF0u) return NW_ERR_ARG;
    NW_TRY(hipSetDevice(ctx->device), "hipSetDevice");
    std::shared_lock<std::shared_mutex> keys(ctx->keys_mu);
    Lease lease(ctx);
    Workspace* ws = lease.ws();
    if (!ws) return NW_ERR_DEVICE;
    hipStream_t st = ws->stream;
    NW_TRY(lease.bind(st, true), "hipStreamWaitEvent");
    uint64_t flen = UINT64_MAX;
    int rc = upload_sig_keys(ctx, ws, msg, len, pk, sig, n, st, &flen);
    if (rc != NW_OK) return rc;
    NW_TRY(ws->ensure(ws->w_out, MSM_PT_WORDS * 4 + 16), "ws point");
    const uint32_t cnt = (uint32_t)n;
    uint32_t* d_bad = nullptr;
    rc = enqueue_msm(ctx, ws, 1, &cnt, n, zseed, batch_index, z_offset, nullptr, ws->w_out.as<uint32_t>(), &d_bad, st,
                     flen);
    if (rc != NW_OK) return rc;
    uint32_t hbad = 0;
    NW_TRY(hipMemcpyAsync(point, ws->w_out.p, NW_POINT_BYTES, hipMemcpyDeviceToHost, st), "D2H point");
    NW_TRY(hipMemcpyAsync(&hbad, d_bad, 4, hipMemcpyDeviceToHost, st), "D2H bad");
    NW_TRY(hipStreamSynchronize(st), "sync");
    lease.synced();
    *bad = hbad ? 1 : 0;
    return NW_OK;
}

int nw_points_sum_is_identity(nw_ctx* ctx, const uint8_t (*points)[NW_POINT_BYTES], size_t k, int* is_identity) {
    if (!ctx || !is_identity || (k && !points)) return NW_ERR_ARG;
    NW_TRY(hipSetDevice(ctx->device), "hipSetDevice");
    // every lease holds the key lock shared: drain_all (exclusive) then never races a lease
    std::shared_lock<std::shared_mutex> keys(ctx->keys_mu);
    Lease lease(ctx);
    Workspace* ws = lease.ws();
    if (!ws) return NW_ERR_DEVICE;
    hipStream_t st = ws->stream;
    NW_TRY(lease.bind(st, true), "hipStreamWaitEvent");
    NW_TRY(ws->ensure(ws->w_misc, k * NW_POINT_BYTES + 64), "ws points");
    if (k) NW_TRY(hipMemcpyAsync(ws->w_misc.p, points, k * NW_POINT_BYTES, hipMemcpyHostToDevice, st), "H2D points");
    uint8_t* d_out = ws->w_misc.as<uint8_t>() + k * NW_POINT_BYTES;
    NW_TRY(launch_msm_points_identity((uint32_t)k, ws->w_misc.as<uint32_t>(), d_out, st), "k_points_identity");
    uint8_t r = 0;
    NW_TRY(hipMemcpyAsync(&r, d_out, 1, hipMemcpyDeviceToHost, st), "D2H");
    NW_TRY(hipStreamSynchronize(st), "sync");
    lease.synced();
    *is_identity = r ? 1 : 0;
    return NW_OK;
}

int nw_verify_certs(nw_ctx* ctx, const nw_cert* certs, size_t ncerts, const uint8_t (*sig)[64],
                    const uint32_t* signer_slot, const uint8_t (*msg)[32], const uint8_t zseed[32], uint64_t cert_base,
                    uint8_t* cert_ok, uint8_t* sig_ok, uint64_t* accepted_stake) {
    if (!ctx || (ncerts && (!certs || !msg))) return NW_ERR_ARG;
    if (!zseed_ok(ctx, zseed)) return NW_ERR_ARG;
    NW_TRY(hipSetDevice(ctx->device), "hipSetDevice");
    size_t nsigs = 0;
    std::vector<uint32_t> first(ncerts), nv(ncerts);
    for (size_t c = 0; c < ncerts; ++c) {
        first[c] = certs[c].first_vote;
        nv[c] = certs[c].n_votes;
        const size_t end = (size_t)certs[c].first_vote + certs[c].n_votes;
        if (end > nsigs) nsigs = end;
    }
    if (nsigs > 0xFFFFFFF0u) return NW_ERR_ARG;
    if (nsigs && (!sig || !signer_slot)) return NW_ERR_ARG;
    if (!ranges_disjoint(first.data(), nv.data(), ncerts)) {
        set_error(ctx, "overlapping certificate vote ranges");
        return NW_ERR_ARG;
    }
    std::shared_lock<std::shared_mutex> keys(ctx->keys_mu);
    for (size_t v = 0; v < nsigs; ++v)
        if (signer_slot[v] >= ctx->nkeys) {
            set_error(ctx, "signer slot out of range (load the committee first)");
            return NW_ERR_ARG;
        }
    if (ncerts == 0) return NW_OK;   // nothing to verify (nsigs is 0 too)
    Lease lease(ctx);
    Workspace* ws = lease.ws();
    if (!ws) return NW_ERR_DEVICE;
    hipStream_t st = ws->stream;
    NW_TRY(lease.bind(st, true), "hipStreamWaitEvent");
    // Every input is staged into pinned memory (see kSmallCallBytes): one D2H for the outputs; small
    // calls also carry the preamble state and go up in one H2D.  The signature array of a large call
    // goes up in 4 MiB chunks, each DMA overlapping the staging memcpy of the next chunk.
    const bool staged = nsigs <= kStagedMaxSigs;   // preamble state rides along: no preamble kernels
    const size_t o_sig = 0, o_signer = align256(o_sig + nsigs * 64), o_first = align256(o_signer + nsigs * 4),
                 o_nv = align256(o_first + ncerts * 4), o_msg = align256(o_nv + ncerts * 4),
                 o_pre = align256(o_msg + ncerts * 32),
                 in_bytes = o_pre + (staged ? prestaged_bytes(nsigs, ncerts) : 0);
    const size_t o_cok = 0, o_stake = align256(ncerts), o_ok = align256(o_stake + ncerts * 8),
                 out_bytes = align256(o_ok + nsigs);
    NW_TRY(ws->ensure(ws->w_io, in_bytes + out_bytes), "ws io");
    NW_TRY(ws->h_io.ensure(in_bytes > out_bytes ? in_bytes : out_bytes), "pinned io");
    uint8_t* h = ws->h_io.bytes();
    uint8_t* d_in = ws->w_io.as<uint8_t>();
    uint8_t* d_out = d_in + in_bytes;
    if (nsigs) std::memcpy(h + o_signer, signer_slot, nsigs * 4);
    std::memcpy(h + o_first, first.data(), ncerts * 4);
    std::memcpy(h + o_nv, nv.data(), ncerts * 4);
    std::memcpy(h + o_msg, msg, ncerts * 32);
    PreStaged pre{};
    if (staged) prestage(h + o_pre, d_in + o_pre, first.data(), nv.data(), ncerts, nsigs, pre);
    const size_t sig_bytes = nsigs * 64;
    if (sig_bytes < kStageChunk) {
        if (sig_bytes) std::memcpy(h + o_sig, sig, sig_bytes);
        NW_TRY(hipMemcpyAsync(d_in, h, in_bytes, hipMemcpyHostToDevice, st), "H2D inputs");
    } else {
        NW_TRY(hipMemcpyAsync(d_in + o_signer, h + o_signer, in_bytes - o_signer, hipMemcpyHostToDevice, st),
               "H2D inputs");
        NW_TRY(staged_h2d(h + o_sig, d_in + o_sig, reinterpret_cast<const uint8_t*>(sig), sig_bytes, st), "H2D sig");
    }
    int rc = enqueue_certs(ctx, ws, ncerts, reinterpret_cast<const uint32_t*>(d_in + o_first),
                           reinterpret_cast<const uint32_t*>(d_in + o_nv), nsigs, d_in + o_sig,
                           reinterpret_cast<const uint32_t*>(d_in + o_signer), 0, d_in + o_msg, nullptr, nullptr,
                           nullptr, zseed, cert_base, 1, d_out + o_cok, nullptr,
                           reinterpret_cast<uint64_t*>(d_out + o_stake), st, sig_ok && nsigs ? d_out + o_ok : nullptr,
                           nullptr, staged ? &pre : nullptr);
    if (rc != NW_OK) return rc;   // the lease synchronizes the stream (the H2D may be in flight)
    // the H2D above has completed in stream order before this copy overwrites the staging buffer
    NW_TRY(hipMemcpyAsync(h, d_out, out_bytes, hipMemcpyDeviceToHost, st), "D2H outputs");
    NW_TRY(hipStreamSynchronize(st), "sync");
    lease.synced();
    if (sig_ok && nsigs) std::memcpy(sig_ok, h + o_ok, nsigs);
    if (cert_ok) std::memcpy(cert_ok, h + o_cok, ncerts);
    if (accepted_stake) std::memcpy(accepted_stake, h + o_stake, ncerts * 8);
    return NW_OK;
}

int nw_verify_batches(nw_ctx* ctx, size_t nb, const uint32_t* first, const uint32_t* nvotes,
                      const uint8_t* const* msg, const size_t* len, const uint32_t* signer_slot,
                      const uint8_t (*sig)[64], const uint8_t zseed[32], uint64_t batch_base, uint8_t* batch_ok,
                      uint8_t* sig_ok) {
    if (!ctx || (nb && (!first || !nvotes))) return NW_ERR_ARG;
    if (!zseed_ok(ctx, zseed)) return NW_ERR_ARG;
    NW_TRY(hipSetDevice(ctx->device), "hipSetDevice");
    size_t nsigs = 0;
    for (size_t b = 0; b < nb; ++b) {
        const size_t end = (size_t)first[b] + nvotes[b];
        if (end > nsigs) nsigs = end;
    }
    if (nsigs > 0xFFFFFFF0u) return NW_ERR_ARG;
    if (nsigs && (!sig || !signer_slot || !msg || !len)) return NW_ERR_ARG;
    if (!ranges_disjoint(first, nvotes, nb)) {
        set_error(ctx, "overlapping batch ranges");
        return NW_ERR_ARG;
    }
    std::shared_lock<std::shared_mutex> keys(ctx->keys_mu);
    for (size_t v = 0; v < nsigs; ++v)
        if (signer_slot[v] >= ctx->nkeys) {
            set_error(ctx, "signer slot out of range (load the keys first)");
            return NW_ERR_ARG;
        }
    Lease lease(ctx);
    Workspace* ws = lease.ws();
    if (!ws) return NW_ERR_DEVICE;
    hipStream_t st = ws->stream;
    NW_TRY(lease.bind(st, true), "hipStreamWaitEvent");
    const size_t total = message_bytes(len, nsigs);
    Stager sg(ws, st);
    NW_TRY(sg.reserve(message_stage_bytes(total, nsigs) + Stager::room(nsigs * 64) + Stager::room(nsigs * 4) +
                      2 * Stager::room(nb * 4)),
           "pinned io");
    int rc = upload_messages(ctx, ws, sg, msg, len, nsigs, total);
    if (rc != NW_OK) return rc;
    NW_TRY(ws->ensure(ws->w_sig, nsigs * 64 + 64), "ws sig");
    NW_TRY(ws->ensure(ws->w_signer, nsigs * 4 + 4), "ws signer");
    NW_TRY(ws->ensure(ws->w_cert_first, nb * 4 + 4), "ws first");
    NW_TRY(ws->ensure(ws->w_cert_n, nb * 4 + 4), "ws n");
    NW_TRY(ws->ensure(ws->w_cert_ok, nb + 16), "ws batch_ok");
    NW_TRY(ws->ensure(ws->w_ok, nsigs + 16), "ws ok");
    NW_TRY(sg.put(ws->w_sig.p, sig, nsigs * 64), "H2D sig");
    NW_TRY(sg.put(ws->w_signer.p, signer_slot, nsigs * 4), "H2D signer");
    NW_TRY(sg.put(ws->w_cert_first.p, first, nb * 4), "H2D first");
    NW_TRY(sg.put(ws->w_cert_n.p, nvotes, nb * 4), "H2D n");
    rc = enqueue_certs(ctx, ws, nb, ws->w_cert_first.as<uint32_t>(), ws->w_cert_n.as<uint32_t>(), nsigs,
                       ws->w_sig.as<uint8_t>(), ws->w_signer.as<uint32_t>(), 1, nullptr, ws->w_msg.as<uint8_t>(),
                       ws->w_msg_off.as<uint64_t>(), ws->w_msg_len.as<uint64_t>(), zseed, batch_base, 1,
                       ws->w_cert_ok.as<uint8_t>(), nullptr, nullptr, st,
                       sig_ok && nsigs ? ws->w_ok.as<uint8_t>() : nullptr);
    if (rc != NW_OK) return rc;
    if (sig_ok && nsigs) NW_TRY(hipMemcpyAsync(sig_ok, ws->w_ok.p, nsigs, hipMemcpyDeviceToHost, st), "D2H sig_ok");
    if (batch_ok && nb) NW_TRY(hipMemcpyAsync(batch_ok, ws->w_cert_ok.p, nb, hipMemcpyDeviceToHost, st), "D2H");
    NW_TRY(hipStreamSynchronize(st), "sync");
    lease.synced();
    return NW_OK;
}

int nw_verify_certs_dev(nw_ctx* ctx, size_t ncerts, const uint32_t* d_cert_first, const uint32_t* d_cert_nvotes,
                        size_t nsigs, const uint8_t* d_sig64, const uint32_t* d_signer_slot, const uint8_t* d_msg32,
                        const uint8_t zseed[32], uint64_t cert_base, uint8_t* d_cert_ok, uint32_t* d_sig_flags,
                        uint64_t* d_accepted_stake, uint32_t* d_status, void* stream) {
    if (!ctx) return NW_ERR_ARG;
    if (!zseed_ok(ctx, zseed)) return NW_ERR_ARG;
    if (ncerts > 0xFFFFFFF0u || nsigs > 0xFFFFFFF0u) return NW_ERR_ARG;
    if ((ncerts && (!d_cert_first || !d_cert_nvotes || !d_msg32)) || (nsigs && (!d_sig64 || !d_signer_slot)))
        return NW_ERR_ARG;
    NW_TRY(hipSetDevice(ctx->device), "hipSetDevice");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    std::shared_lock<std::shared_mutex> keys(ctx->keys_mu);
    if (nsigs && ctx->nkeys == 0) {   // every slot is out of range, and the kernels have no table to clamp to
        set_error(ctx, "nw_verify_certs_dev: no committee loaded (signer slots outside the empty key cache)");
        return NW_ERR_ARG;
    }
    Lease lease(ctx, st);
    Workspace* ws = lease.ws();
    if (!ws) return NW_ERR_DEVICE;
    NW_TRY(lease.bind(st, false), "hipStreamWaitEvent");
    // Input validation on the device (the inputs are device-resident) inside the batch preamble
    // (k_expand_count): with d_status it is written there in stream order; without it the call waits
    // for the check and returns NW_ERR_ARG before any verification is enqueued.  Every kernel also
    // clamps the inputs, so invalid inputs never fault.
    int rc = enqueue_certs(ctx, ws, ncerts, d_cert_first, d_cert_nvotes, nsigs, d_sig64, d_signer_slot, 0, d_msg32,
                           nullptr, nullptr, nullptr, zseed, cert_base, 1, d_cert_ok, d_sig_flags, d_accepted_stake,
                           st, nullptr, d_status, nullptr, d_status == nullptr);
    if (rc == NW_ERR_ARG) {
        lease.synced();
        return rc;
    }
    NW_TRY(lease.finish(), "hipEventRecord");
    return rc;
}

int nw_sha512_many_dev(nw_ctx* ctx, const uint8_t* d_base, const uint64_t* d_off, const uint64_t* d_len, size_t n,
                       uint8_t* d_out64, void* stream) {
    if (!ctx || (n && (!d_base || !d_off || !d_len || !d_out64))) return NW_ERR_ARG;
    if (n > 0xFFFFFFF0u) return NW_ERR_ARG;
    NW_TRY(hipSetDevice(ctx->device), "hipSetDevice");
    NW_TRY(launch_sha512_many((uint32_t)n, d_base, d_off, d_len, d_out64, reinterpret_cast<hipStream_t>(stream)),
           "k_sha512_many");
    return NW_OK;
}

int nw_sha512_many(nw_ctx* ctx, const uint8_t* base, const uint64_t* off, const uint64_t* len, size_t n,
                   uint8_t (*out)[64]) {
    if (!ctx || (n && (!off || !len || !out))) return NW_ERR_ARG;
    if (n == 0) return NW_OK;
    if (n > 0xFFFFFFF0u) return NW_ERR_ARG;
    NW_TRY(hipSetDevice(ctx->device), "hipSetDevice");
    // upload only the referenced span
    uint64_t lo = UINT64_MAX, hi = 0;
    for (size_t i = 0; i < n; ++i) {
        if (off[i] < lo) lo = off[i];
        if (off[i] + len[i] > hi) hi = off[i] + len[i];
    }
    if (hi < lo) hi = lo;
    if (hi > lo && !base) return NW_ERR_ARG;
    std::vector<uint64_t> roff(n);
    for (size_t i = 0; i < n; ++i) roff[i] = off[i] - lo;
    const size_t span = (size_t)(hi - lo);
    std::shared_lock<std::shared_mutex> keys(ctx->keys_mu);   // see nw_points_sum_is_identity
    Lease lease(ctx);
    Workspace* ws = lease.ws();
    if (!ws) return NW_ERR_DEVICE;
    hipStream_t st = ws->stream;
    NW_TRY(lease.bind(st, true), "hipStreamWaitEvent");
    NW_TRY(ws->ensure(ws->w_msg, span + 16), "ws msg");
    NW_TRY(ws->ensure(ws->w_msg_off, n * 8), "ws off");
    NW_TRY(ws->ensure(ws->w_msg_len, n * 8), "ws len");
    NW_TRY(ws->ensure(ws->w_out, n * 64), "ws out");
    // everything through the pinned buffer (see kSmallCallBytes): offsets, lengths, then the data
    const size_t o_off = 0, o_len = align256(n * 8), o_data = o_len + align256(n * 8);
    NW_TRY(ws->h_io.ensure(std::max(o_data + span, n * 64)), "pinned io");
    uint8_t* h = ws->h_io.bytes();
    std::memcpy(h + o_off, roff.data(), n * 8);
    std::memcpy(h + o_len, len, n * 8);
    NW_TRY(hipMemcpyAsync(ws->w_msg_off.p, h + o_off, n * 8, hipMemcpyHostToDevice, st), "H2D off");
    NW_TRY(hipMemcpyAsync(ws->w_msg_len.p, h + o_len, n * 8, hipMemcpyHostToDevice, st), "H2D len");
    if (span) NW_TRY(staged_h2d(h + o_data, ws->w_msg.as<uint8_t>(), base + lo, span, st), "H2D data");
    NW_TRY(launch_sha512_many((uint32_t)n, ws->w_msg.as<uint8_t>(), ws->w_msg_off.as<uint64_t>(),
                              ws->w_msg_len.as<uint64_t>(), ws->w_out.as<uint8_t>(), st),
           "k_sha512_many");
    // the uploads have completed in stream order before this copy reuses the pinned buffer
    NW_TRY(hipMemcpyAsync(h, ws->w_out.p, n * 64, hipMemcpyDeviceToHost, st), "D2H digests");
    NW_TRY(hipStreamSynchronize(st), "sync");
    lease.synced();
    std::memcpy(out, h, n * 64);
    return NW_OK;
}

int nw_sha512(nw_ctx* ctx, const uint8_t* data, size_t len, uint8_t out[64]) {
    const uint64_t off = 0, ln = len;
    static const uint8_t empty[1] = {0};
    return nw_sha512_many(ctx, data ? data : empty, &off, &ln, 1, reinterpret_cast<uint8_t(*)[64]>(out));
}

// Asynchronous batch digest (the worker's Processor loop, worker/src/processor.rs:63-97).  The job
// owns a workspace lease from submit to wait, so its pinned staging buffer (the messages in, the
// digests out) is never reused under it; it does not mark the workspace pending and holds no key
// lock (a digest reads no key table, so committee loads need not wait for it).  The messages are
// packed into the pinned buffer at 16-byte aligned offsets (a worker's batches are fresh buffers
// on every call: see kSmallCallBytes for why nothing is copied from pageable memory), and every
// 4 MiB packed is sent at once, so the DMAs overlap the packing.
int nw_sha512_many_async(nw_ctx* ctx, const uint8_t* const* msg, const size_t* len, size_t n, uint8_t (*out)[64],
                         nw_job** job) {
    if (!ctx || !job || (n && (!msg || !len || !out))) return NW_ERR_ARG;
    *job = nullptr;
    if (n > 0xFFFFFFF0u) return NW_ERR_ARG;
    for (size_t i = 0; i < n; ++i)
        if (len[i] && !msg[i]) return NW_ERR_ARG;
    auto j = std::make_unique<nw_job>();
    j->out = reinterpret_cast<uint8_t*>(out);
    j->n = n;
    if (n == 0) {
        *job = j.release();
        return NW_OK;
    }
    NW_TRY(hipSetDevice(ctx->device), "hipSetDevice");
    if (ctx->async_jobs.fetch_add(1) >= kMaxAsyncJobs) {
        ctx->async_jobs.fetch_sub(1);
        set_error(ctx, "nw_sha512_many_async: too many unwaited jobs (limit 32; wait for one first)");
        return NW_ERR_NOMEM;
    }
    j->inflight = &ctx->async_jobs;
    std::vector<uint64_t> off(n);
    size_t total = 0;
    for (size_t i = 0; i < n; ++i) {
        off[i] = total;
        total += (len[i] + 15) & ~(size_t)15;
    }
    const size_t o_off = 0, o_len = align256(n * 8), o_msg = o_len + align256(n * 8), o_out = o_msg + align256(total);
    j->lease = std::make_unique<Lease>(ctx, nullptr, o_out + n * 64);
    Workspace* ws = j->lease->ws();
    if (!ws) return NW_ERR_DEVICE;
    hipStream_t st = ws->stream;
    NW_TRY(j->lease->bind(st, true), "hipStreamWaitEvent");
    j->o_out = o_out;
    NW_TRY(ws->h_io.ensure(o_out + n * 64), "pinned io");
    NW_TRY(ws->ensure(ws->w_msg, total + 16), "ws msg");
    NW_TRY(ws->ensure(ws->w_msg_off, n * 8), "ws off");
    NW_TRY(ws->ensure(ws->w_msg_len, n * 8), "ws len");
    NW_TRY(ws->ensure(ws->w_out, n * 64), "ws out");
    uint8_t* h = ws->h_io.bytes();
    std::memcpy(h + o_off, off.data(), n * 8);
    for (size_t i = 0; i < n; ++i) reinterpret_cast<uint64_t*>(h + o_len)[i] = len[i];
    NW_TRY(hipMemcpyAsync(ws->w_msg_off.p, h + o_off, n * 8, hipMemcpyHostToDevice, st), "H2D off");
    NW_TRY(hipMemcpyAsync(ws->w_msg_len.p, h + o_len, n * 8, hipMemcpyHostToDevice, st), "H2D len");
    uint8_t* d_msg = ws->w_msg.as<uint8_t>();
    // chunks of whole messages, each closed once it holds >= kStageChunk bytes
    std::vector<size_t> cb{0}, cm{0};   // chunk byte starts, chunk first-message indices
    for (size_t i = 0; i < n; ++i) {
        const size_t packed = i + 1 < n ? off[i + 1] : total;
        if (packed - cb.back() >= kStageChunk || (i + 1 == n && packed > cb.back())) {
            cb.push_back(packed);
            cm.push_back(i + 1);
        }
    }
    if (cb.size() > 1) {
        NW_TRY(stage_chunks(cb.size() - 1, cb.data(),
                            [&](size_t c) {
                                for (size_t i = cm[c]; i < cm[c + 1]; ++i)
                                    if (len[i]) std::memcpy(h + o_msg + off[i], msg[i], len[i]);
                            },
                            h + o_msg, d_msg, st),
               "H2D messages");
    }
    NW_TRY(launch_sha512_many((uint32_t)n, d_msg, ws->w_msg_off.as<uint64_t>(), ws->w_msg_len.as<uint64_t>(),
                              ws->w_out.as<uint8_t>(), st),
           "k_sha512_many");
    NW_TRY(hipMemcpyAsync(h + o_out, ws->w_out.p, n * 64, hipMemcpyDeviceToHost, st), "D2H digests");
    NW_TRY(hipEventRecord(ws->done, st), "hipEventRecord");
    *job = j.release();
    return NW_OK;
}

int nw_job_done(nw_job* job) {
    if (!job) return NW_ERR_ARG;
    if (!job->lease) return 1;
    const hipError_t e = hipEventQuery(job->lease->ws()->done);
    if (e == hipSuccess) return 1;
    return e == hipErrorNotReady ? 0 : -NW_ERR_DEVICE;
}

int nw_job_wait(nw_job* job) {
    if (!job) return NW_ERR_ARG;
    std::unique_ptr<nw_job> own(job);
    if (!own->lease) return NW_OK;
    Workspace* ws = own->lease->ws();
    const hipError_t e = hipEventSynchronize(ws->done);
    if (e != hipSuccess) {
        tl_last_error = std::string("nw_job_wait: ") + hipGetErrorString(e);
        return NW_ERR_DEVICE;   // the lease synchronizes its stream on release
    }
    std::memcpy(own->out, ws->h_io.bytes() + own->o_out, own->n * 64);
    own->lease->synced();
    return NW_OK;
}

int nw_sign_many_dev(nw_ctx* ctx, const uint8_t* d_seed32, const uint8_t* d_msgs, size_t msg_len, size_t n,
                     uint8_t* d_pk32, uint8_t* d_sig64, void* stream) {
    if (!ctx || (msg_len != 8 && msg_len != 32)) return NW_ERR_ARG;
    if (n > 0xFFFFFFF0u || (n && (!d_seed32 || !d_msgs))) return NW_ERR_ARG;
    NW_TRY(hipSetDevice(ctx->device), "hipSetDevice");
    std::shared_lock<std::shared_mutex> keys(ctx->keys_mu);   // reads the basepoint table
    NW_TRY(launch_sign((uint32_t)n, (int)(msg_len / 4), reinterpret_cast<const uint32_t*>(d_seed32),
                       reinterpret_cast<const uint32_t*>(d_msgs), ctx->d_btab, reinterpret_cast<uint32_t*>(d_pk32),
                       reinterpret_cast<uint32_t*>(d_sig64), reinterpret_cast<hipStream_t>(stream)),
           "k_sign");
    return NW_OK;
}

int nw_sign_many(nw_ctx* ctx, const uint8_t (*seed)[32], const uint8_t* msgs, size_t msg_len, size_t n,
                 uint8_t (*pk)[32], uint8_t (*sig)[64]) {
    if (!ctx || (msg_len != 8 && msg_len != 32) || (n && (!seed || !msgs))) return NW_ERR_ARG;
    if (n == 0) return NW_OK;
    if (n > 0xFFFFFFF0u) return NW_ERR_ARG;
    NW_TRY(hipSetDevice(ctx->device), "hipSetDevice");
    std::shared_lock<std::shared_mutex> keys(ctx->keys_mu);   // see nw_points_sum_is_identity
    Lease lease(ctx);
    Workspace* ws = lease.ws();
    if (!ws) return NW_ERR_DEVICE;
    hipStream_t st = ws->stream;
    NW_TRY(lease.bind(st, true), "hipStreamWaitEvent");
    NW_TRY(ws->ensure(ws->w_misc, n * 32 + n * msg_len + 16), "ws misc");
    NW_TRY(ws->ensure(ws->w_out, n * 96 + 16), "ws out");
    uint8_t* d_seed = ws->w_misc.as<uint8_t>();
    uint8_t* d_msg = d_seed + n * 32;
    uint8_t* d_pk = ws->w_out.as<uint8_t>();
    uint8_t* d_sig = d_pk + n * 32;
    NW_TRY(hipMemcpyAsync(d_seed, seed, n * 32, hipMemcpyHostToDevice, st), "H2D seed");
    NW_TRY(hipMemcpyAsync(d_msg, msgs, n * msg_len, hipMemcpyHostToDevice, st), "H2D msg");
    NW_TRY(launch_sign((uint32_t)n, (int)(msg_len / 4), reinterpret_cast<const uint32_t*>(d_seed),
                       reinterpret_cast<const uint32_t*>(d_msg), ctx->d_btab, reinterpret_cast<uint32_t*>(d_pk),
                       reinterpret_cast<uint32_t*>(d_sig), st),
           "k_sign");
    if (pk) NW_TRY(hipMemcpyAsync(pk, d_pk, n * 32, hipMemcpyDeviceToHost, st), "D2H pk");
    if (sig) NW_TRY(hipMemcpyAsync(sig, d_sig, n * 64, hipMemcpyDeviceToHost, st), "D2H sig");
    NW_TRY(hipStreamSynchronize(st), "sync");
    lease.synced();
    return NW_OK;
}

}  // extern "C"
