// C-ABI host layer of libnwcrypto (include/nwcrypto.h): device memory, the key cache, workspace,
// and the launch sequences.  No CPU compute path: every verdict and digest comes from the GPU.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "nw_kernels.h"
#include "nw_point.h"

using namespace nw;

namespace {

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

}  // namespace

struct nw_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    uint32_t finish_k = FINISH_K;   // k_finish signatures per lane
    std::mutex mu;
    std::string last_error;
    // basepoint comb
    uint32_t* d_btab = nullptr;
    // key cache
    size_t max_keys = 0;          // 0: derived from the HBM budget once the window is fixed
    bool max_keys_user = false;
    int key_window = 0;           // 0: not yet decided (first load)
    size_t key_words = 0;         // u32 words per key table
    size_t nkeys = 0, key_cap = 0;
    uint32_t* d_keys_raw = nullptr;
    uint32_t* d_key_info = nullptr;
    uint32_t* d_stake = nullptr;
    uint32_t* d_key_tab = nullptr;
    std::unordered_map<std::string, uint32_t> slot_of;
    std::vector<uint32_t> h_stake;
    // measurement: (start, stop) event pairs around k_verify launches
    bool prof_on = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> prof_events;
    size_t prof_used = 0;
    uint64_t prof_sigs = 0;
    // workspace
    DevBuf w_bases, w_sig, w_signer, w_sig_cert, w_cert_first, w_cert_n, w_msg, w_msg_off, w_msg_len,
        w_flags, w_slow_count, w_slow_list, w_slow_slot, w_slow_buf, w_cert_ok, w_stake_out, w_ok, w_misc,
        w_out, w_pbuf, w_pre, w_counts, w_cursor, w_perm, w_io;
    HostBuf h_io;
};

namespace {

int fail(nw_ctx* c, hipError_t e, const char* what) {
    if (c) {
        c->last_error = std::string(what) + ": " + hipGetErrorString(e);
    }
    return e == hipErrorOutOfMemory ? NW_ERR_NOMEM : NW_ERR_DEVICE;
}

#define NW_TRY(expr, what)                              \
    do {                                                \
        hipError_t e_ = (expr);                         \
        if (e_ != hipSuccess) return fail(ctx, e_, what); \
    } while (0)

// Basepoint encoding (y = 4/5, x even).
const uint8_t kBaseEnc[32] = {0x58, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66,
                              0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66,
                              0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66};

// k_finish signatures per lane (NW_FK overrides it for tuning; 1..FINISH_K).  Measured on MI355X:
// splitting a batch into chunks so k_finish of one chunk overlaps k_verify of the next on a second
// stream was slower (623 vs 712 M sigs/s at C2: the co-running k_finish waves take VGPR slots from
// the VALU-bound k_verify and every chunk pays a tail), so a batch is one k_verify + one k_finish.
uint32_t finish_k() {
    const char* e = std::getenv("NW_FK");
    const long k = e ? std::strtol(e, nullptr, 10) : 0;
    return k >= 1 && k <= FINISH_K ? (uint32_t)k : (uint32_t)FINISH_K;
}

constexpr size_t KEY_CACHE_BUDGET = 160ull << 30;  // bytes of HBM for key tables by default (of 288 GB)
constexpr size_t kGroupMinSigs = 16384;            // group signatures by signer above this batch size

// Key comb window, fixed at the first load.  Auto (0): a conservative choice that leaves room for
// keys added later.  Committee mode (-1): the first load IS the committee; take the widest window
// whose tables for it fit the key budget with 25% headroom (fewest additions per signature).
int committee_window(size_t n, size_t budget) {
    for (int w : {20, 16, 12}) {
        const double need = 1.25 * (double)n * (double)comb_words(w) * 4.0;
        if (need <= (double)budget) return w;
    }
    return 8;
}

void fix_window(nw_ctx* ctx, size_t first_load) {
    const size_t budget = ctx->max_keys_user ? (size_t)-1 : KEY_CACHE_BUDGET;
    if (ctx->key_window == -1) ctx->key_window = committee_window(first_load, budget);
    if (ctx->key_window == 0) ctx->key_window = first_load <= 384 ? 16 : (first_load <= 12288 ? 12 : 8);
    ctx->key_words = comb_words(ctx->key_window);
    if (!ctx->max_keys_user) ctx->max_keys = KEY_CACHE_BUDGET / (ctx->key_words * 4);
}

int grow_keys(nw_ctx* ctx, size_t need) {
    if (need <= ctx->key_cap) return NW_OK;
    if (need > ctx->max_keys) {
        ctx->last_error = "key cache capacity exceeded (nw_opts.max_keys)";
        return NW_ERR_NOMEM;
    }
    size_t cap = ctx->key_cap ? ctx->key_cap : 64;
    while (cap < need) cap *= 2;
    if (cap > ctx->max_keys) cap = ctx->max_keys;
    uint32_t *raw = nullptr, *info = nullptr, *stake = nullptr, *tab = nullptr;
    NW_TRY(hipMalloc(&raw, cap * 32), "hipMalloc(keys_raw)");
    NW_TRY(hipMalloc(&info, cap * 4), "hipMalloc(key_info)");
    NW_TRY(hipMalloc(&stake, cap * 4), "hipMalloc(stake)");
    NW_TRY(hipMalloc(&tab, cap * ctx->key_words * 4), "hipMalloc(key_tab)");
    if (ctx->nkeys) {
        NW_TRY(hipMemcpyAsync(raw, ctx->d_keys_raw, ctx->nkeys * 32, hipMemcpyDeviceToDevice, ctx->stream), "copy");
        NW_TRY(hipMemcpyAsync(info, ctx->d_key_info, ctx->nkeys * 4, hipMemcpyDeviceToDevice, ctx->stream), "copy");
        NW_TRY(hipMemcpyAsync(stake, ctx->d_stake, ctx->nkeys * 4, hipMemcpyDeviceToDevice, ctx->stream), "copy");
        NW_TRY(hipMemcpyAsync(tab, ctx->d_key_tab, ctx->nkeys * ctx->key_words * 4, hipMemcpyDeviceToDevice,
                              ctx->stream),
               "copy");
        NW_TRY(hipStreamSynchronize(ctx->stream), "sync");
        (void)hipFree(ctx->d_keys_raw);
        (void)hipFree(ctx->d_key_info);
        (void)hipFree(ctx->d_stake);
        (void)hipFree(ctx->d_key_tab);
    }
    ctx->d_keys_raw = raw;
    ctx->d_key_info = info;
    ctx->d_stake = stake;
    ctx->d_key_tab = tab;
    ctx->key_cap = cap;
    return NW_OK;
}

// Build tables for keys [k0, k0 + nk) whose raw bytes are already in d_keys_raw.
int build_keys(nw_ctx* ctx, uint32_t* d_raw, uint32_t* d_info, uint32_t* d_tab, size_t nk, int window) {
    // keys per launch: bounds the bases scratch and keeps a launch near 16M chunk threads
    const size_t chunk = window >= 24 ? 1 : (window == 20 ? 16 : (window == 16 ? 256 : 4096));
    const size_t words = comb_words(window);
    for (size_t s = 0; s < nk; s += chunk) {
        const size_t m = nk - s < chunk ? nk - s : chunk;
        NW_TRY(ctx->w_bases.ensure(m * comb_pos(window) * 40 * 4), "hipMalloc(bases)");
        NW_TRY(launch_key_prep((uint32_t)m, d_raw + s * 8, d_info + s, ctx->w_bases.as<uint32_t>(), d_tab + s * words,
                               window, ctx->stream),
               "k_key_prep/k_comb_build");
    }
    return NW_OK;
}

// Map keys to cache slots, loading unknown keys (table build on the GPU).
int ensure_slots(nw_ctx* ctx, const uint8_t (*pk)[32], const uint32_t* stake, size_t n, uint32_t* slots) {
    std::vector<uint32_t> new_idx;
    std::vector<uint8_t> new_raw;
    std::unordered_map<std::string, uint32_t> pending;
    for (size_t i = 0; i < n; ++i) {
        std::string k(reinterpret_cast<const char*>(pk[i]), 32);
        auto it = ctx->slot_of.find(k);
        if (it != ctx->slot_of.end()) {
            slots[i] = it->second;
            if (stake) {
                ctx->h_stake[it->second] = stake[i];
                new_idx.push_back(it->second);   // stake refresh only
            }
            continue;
        }
        auto pit = pending.find(k);
        if (pit != pending.end()) {
            slots[i] = pit->second;
            continue;
        }
        const uint32_t slot = (uint32_t)(ctx->nkeys + pending.size());
        pending.emplace(k, slot);
        slots[i] = slot;
        new_raw.insert(new_raw.end(), pk[i], pk[i] + 32);
        ctx->h_stake.push_back(stake ? stake[i] : 0u);
    }
    const size_t add = pending.size();
    if (add && ctx->key_window <= 0) fix_window(ctx, add);
    if (add) {
        int rc = grow_keys(ctx, ctx->nkeys + add);
        if (rc != NW_OK) {
            ctx->h_stake.resize(ctx->nkeys);
            return rc;
        }
        const size_t k0 = ctx->nkeys;
        NW_TRY(hipMemcpyAsync(ctx->d_keys_raw + k0 * 8, new_raw.data(), add * 32, hipMemcpyHostToDevice, ctx->stream),
               "H2D keys");
        rc = build_keys(ctx, ctx->d_keys_raw + k0 * 8, ctx->d_key_info + k0, ctx->d_key_tab + k0 * ctx->key_words,
                        add, ctx->key_window);
        if (rc != NW_OK) return rc;
        for (auto& kv : pending) ctx->slot_of.emplace(kv.first, kv.second);
        ctx->nkeys += add;
    }
    if (add || !new_idx.empty()) {
        NW_TRY(hipMemcpyAsync(ctx->d_stake, ctx->h_stake.data(), ctx->nkeys * 4, hipMemcpyHostToDevice, ctx->stream),
               "H2D stake");
        NW_TRY(hipStreamSynchronize(ctx->stream), "sync(committee)");
    }
    return NW_OK;
}

void fill_zseed(uint32_t out[8], const uint8_t* zseed) {
    if (!zseed) {
        for (int k = 0; k < 8; ++k) out[k] = 0;
        return;
    }
    std::memcpy(out, zseed, 32);
}

// Enqueue the certificate pipeline on device buffers.
int enqueue_certs(nw_ctx* ctx, size_t ncerts, const uint32_t* d_first, const uint32_t* d_nv, size_t nsigs,
                  const uint8_t* d_sig, const uint32_t* d_signer, int msgmode, const uint8_t* d_msg32,
                  const uint8_t* d_msg_base, const uint64_t* d_msg_off, const uint64_t* d_msg_len,
                  const uint8_t* zseed, uint64_t cert_base, uint32_t batch_mode, uint8_t* d_cert_ok,
                  uint32_t* d_flags_user, uint64_t* d_stake_out, hipStream_t st) {
    uint32_t* d_flags = d_flags_user;
    if (!d_flags) {
        NW_TRY(ctx->w_flags.ensure(nsigs * 4 + 4), "ws flags");
        d_flags = ctx->w_flags.as<uint32_t>();
    }
    NW_TRY(ctx->w_sig_cert.ensure(nsigs * 4 + 4), "ws sig_cert");
    NW_TRY(ctx->w_slow_count.ensure(16), "ws slow_count");
    NW_TRY(ctx->w_slow_list.ensure(nsigs * 4 + 4), "ws slow_list");
    NW_TRY(ctx->w_slow_slot.ensure(nsigs * 4 + 4), "ws slow_slot");
    if (batch_mode) NW_TRY(ctx->w_slow_buf.ensure(nsigs * (size_t)SLOW_WORDS * 4 + 4), "ws slow_buf");
    NW_TRY(ctx->w_pbuf.ensure(nsigs * (size_t)PBUF_WORDS * 4 + 16), "ws pbuf");
    NW_TRY(ctx->w_pre.ensure(nsigs * 40 + 16), "ws pre");
    // votes not covered by any certificate map to certificate 0 (never out of range)
    NW_TRY(hipMemsetAsync(ctx->w_sig_cert.p, 0, nsigs * 4 + 4, st), "memset sig_cert");
    NW_TRY(launch_expand_certs((uint32_t)ncerts, d_first, d_nv, ctx->w_sig_cert.as<uint32_t>(),
                               ctx->w_slow_count.as<uint32_t>(), st),
           "k_expand_certs");   // also zeroes the slow-path counter

    VerifyParams vp{};
    vp.n = (uint32_t)nsigs;
    vp.batch_mode = batch_mode;
    vp.sig = d_sig;
    vp.signer = d_signer;
    vp.sig_cert = ctx->w_sig_cert.as<uint32_t>();
    vp.cert_first = d_first;
    vp.cert_msg = d_msg32;
    vp.msg_base = d_msg_base;
    vp.msg_off = d_msg_off;
    vp.msg_len = d_msg_len;
    vp.cert_base = cert_base;
    vp.keys_raw = ctx->d_keys_raw;
    vp.key_info = ctx->d_key_info;
    vp.key_tab = ctx->d_key_tab;
    vp.btab = ctx->d_btab;
    fill_zseed(vp.zseed, zseed);
    vp.flags = d_flags;
    vp.slow_count = ctx->w_slow_count.as<uint32_t>();
    vp.slow_list = ctx->w_slow_list.as<uint32_t>();
    vp.slow_slot = ctx->w_slow_slot.as<uint32_t>();
    vp.slow_buf = ctx->w_slow_buf.as<uint32_t>();
    vp.pbuf = ctx->w_pbuf.as<uint32_t>();
    vp.pre = ctx->w_pre.as<uint32_t>();
    vp.perm = nullptr;
    if (nsigs >= kGroupMinSigs && ctx->nkeys > 1) {
        NW_TRY(ctx->w_counts.ensure(ctx->nkeys * 4 + 16), "ws counts");
        NW_TRY(ctx->w_cursor.ensure(ctx->nkeys * 4 + 16), "ws cursor");
        NW_TRY(ctx->w_perm.ensure(nsigs * 4 + 16), "ws perm");
        NW_TRY(launch_group_by_signer((uint32_t)nsigs, (uint32_t)ctx->nkeys, d_signer, ctx->w_counts.as<uint32_t>(),
                                      ctx->w_cursor.as<uint32_t>(), ctx->w_perm.as<uint32_t>(), st),
               "signer grouping");
        vp.perm = ctx->w_perm.as<uint32_t>();
    }
    vp.g0 = 0;
    vp.gn = (uint32_t)nsigs;
    vp.fk = ctx->finish_k;
    hipEvent_t ev_stop = nullptr;
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
    NW_TRY(launch_verify(vp, msgmode, ctx->key_window, st), "k_verify");
    if (ev_stop) NW_TRY(hipEventRecord(ev_stop, st), "hipEventRecord");   // brackets k_verify alone
    NW_TRY(launch_finish(vp, st), "k_finish");
    if (!batch_mode) return NW_OK;

    NW_TRY(launch_slow(vp, msgmode, ctx->key_window, (uint32_t)nsigs, st), "k_slow_sig");

    FinalizeParams fp{};
    fp.ncerts = (uint32_t)ncerts;
    fp.cert_first = d_first;
    fp.cert_n = d_nv;
    fp.flags = d_flags;
    fp.signer = d_signer;
    fp.stake = ctx->d_stake;
    fp.slow_slot = vp.slow_slot;
    fp.slow_buf = vp.slow_buf;
    fp.cert_ok = d_cert_ok;
    fp.accepted_stake = d_stake_out;
    NW_TRY(launch_finalize(fp, st), "k_cert_finalize");
    return NW_OK;
}

// Pack per-signature messages into one device buffer (MSGMODE 1).
int upload_messages(nw_ctx* ctx, const uint8_t* const* msg, const size_t* len, size_t n) {
    std::vector<uint64_t> off(n), ln(n);
    size_t total = 0;
    for (size_t i = 0; i < n; ++i) {
        off[i] = total;
        ln[i] = len[i];
        total += len[i];
    }
    std::vector<uint8_t> packed(total + 8);
    for (size_t i = 0; i < n; ++i)
        if (len[i]) std::memcpy(packed.data() + off[i], msg[i], len[i]);
    NW_TRY(ctx->w_msg.ensure(total + 8), "ws msg");
    NW_TRY(ctx->w_msg_off.ensure(n * 8 + 8), "ws msg_off");
    NW_TRY(ctx->w_msg_len.ensure(n * 8 + 8), "ws msg_len");
    NW_TRY(hipMemcpyAsync(ctx->w_msg.p, packed.data(), total + 8, hipMemcpyHostToDevice, ctx->stream), "H2D msg");
    NW_TRY(hipMemcpyAsync(ctx->w_msg_off.p, off.data(), n * 8, hipMemcpyHostToDevice, ctx->stream), "H2D off");
    NW_TRY(hipMemcpyAsync(ctx->w_msg_len.p, ln.data(), n * 8, hipMemcpyHostToDevice, ctx->stream), "H2D len");
    return NW_OK;
}

// Shared body of strict_many / verify_batch: every signature in one "certificate" 0.
int run_generic(nw_ctx* ctx, const uint8_t* const* msg, const size_t* len, const uint8_t (*pk)[32],
                const uint8_t (*sig)[64], size_t n, const uint8_t* zseed, uint64_t batch_index, uint32_t batch_mode,
                uint8_t* ok_out, uint8_t* verdict_out) {
    std::vector<uint32_t> slots(n);
    int rc = ensure_slots(ctx, pk, nullptr, n, slots.data());
    if (rc != NW_OK) return rc;
    rc = upload_messages(ctx, msg, len, n);
    if (rc != NW_OK) return rc;
    NW_TRY(ctx->w_sig.ensure(n * 64), "ws sig");
    NW_TRY(ctx->w_signer.ensure(n * 4), "ws signer");
    NW_TRY(ctx->w_cert_first.ensure(16), "ws first");
    NW_TRY(ctx->w_cert_n.ensure(16), "ws n");
    NW_TRY(ctx->w_cert_ok.ensure(16), "ws cert_ok");
    NW_TRY(ctx->w_ok.ensure(n + 16), "ws ok");
    const uint32_t first = 0, nv = (uint32_t)n;
    NW_TRY(hipMemcpyAsync(ctx->w_sig.p, sig, n * 64, hipMemcpyHostToDevice, ctx->stream), "H2D sig");
    NW_TRY(hipMemcpyAsync(ctx->w_signer.p, slots.data(), n * 4, hipMemcpyHostToDevice, ctx->stream), "H2D signer");
    NW_TRY(hipMemcpyAsync(ctx->w_cert_first.p, &first, 4, hipMemcpyHostToDevice, ctx->stream), "H2D first");
    NW_TRY(hipMemcpyAsync(ctx->w_cert_n.p, &nv, 4, hipMemcpyHostToDevice, ctx->stream), "H2D n");
    rc = enqueue_certs(ctx, 1, ctx->w_cert_first.as<uint32_t>(), ctx->w_cert_n.as<uint32_t>(), n,
                       ctx->w_sig.as<uint8_t>(), ctx->w_signer.as<uint32_t>(), 1, nullptr, ctx->w_msg.as<uint8_t>(),
                       ctx->w_msg_off.as<uint64_t>(), ctx->w_msg_len.as<uint64_t>(), zseed, batch_index, batch_mode,
                       ctx->w_cert_ok.as<uint8_t>(), nullptr, nullptr, ctx->stream);
    if (rc != NW_OK) return rc;
    if (ok_out) {
        NW_TRY(launch_flags_to_ok((uint32_t)n, ctx->w_flags.as<uint32_t>(), ctx->w_ok.as<uint8_t>(), ctx->stream),
               "k_flags_to_ok");
        NW_TRY(hipMemcpyAsync(ok_out, ctx->w_ok.p, n, hipMemcpyDeviceToHost, ctx->stream), "D2H ok");
    }
    if (verdict_out) NW_TRY(hipMemcpyAsync(verdict_out, ctx->w_cert_ok.p, 1, hipMemcpyDeviceToHost, ctx->stream), "D2H");
    NW_TRY(hipStreamSynchronize(ctx->stream), "sync");
    return NW_OK;
}

}  // namespace

extern "C" {

const char* nw_version(void) { return "nwcrypto 0.1 gfx950 " __DATE__; }

int nw_ctx_create(nw_ctx** out, const nw_opts* opts) {
    if (!out) return NW_ERR_ARG;
    *out = nullptr;
    nw_ctx* ctx = new nw_ctx();
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev == 0) {
        delete ctx;
        return NW_ERR_DEVICE;
    }
    int dev = opts && opts->device >= 0 ? opts->device : -1;
    if (dev < 0) {
        e = hipGetDevice(&dev);
        if (e != hipSuccess) {
            delete ctx;
            return NW_ERR_DEVICE;
        }
    }
    if (dev >= ndev) {
        delete ctx;
        return NW_ERR_ARG;
    }
    ctx->device = dev;
    ctx->finish_k = finish_k();
    if (opts && opts->max_keys) {
        ctx->max_keys = opts->max_keys;
        ctx->max_keys_user = true;
    }
    if (opts && opts->key_window) {
        if (opts->key_window != -1 && opts->key_window != 8 && opts->key_window != 12 && opts->key_window != 16 &&
            opts->key_window != 20) {
            delete ctx;
            return NW_ERR_ARG;
        }
        ctx->key_window = opts->key_window;
        if (ctx->key_window > 0) fix_window(ctx, 0);
    }
    if (hipSetDevice(dev) != hipSuccess || hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
        delete ctx;
        return NW_ERR_DEVICE;
    }
    // basepoint comb (one "key" = B)
    uint32_t* d_braw = nullptr;
    uint32_t* d_binfo = nullptr;
    if (hipMalloc(&ctx->d_btab, comb_words(B_WINDOW) * 4) != hipSuccess || hipMalloc(&d_braw, 32) != hipSuccess ||
        hipMalloc(&d_binfo, 16) != hipSuccess) {
        nw_ctx_destroy(ctx);
        return NW_ERR_NOMEM;
    }
    int rc = NW_OK;
    if (hipMemcpy(d_braw, kBaseEnc, 32, hipMemcpyHostToDevice) != hipSuccess) rc = NW_ERR_DEVICE;
    if (rc == NW_OK) rc = build_keys(ctx, d_braw, d_binfo, ctx->d_btab, 1, B_WINDOW);
    if (rc == NW_OK && hipStreamSynchronize(ctx->stream) != hipSuccess) rc = NW_ERR_DEVICE;
    (void)hipFree(d_braw);
    (void)hipFree(d_binfo);
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
    for (DevBuf* b : {&ctx->w_bases, &ctx->w_sig, &ctx->w_signer, &ctx->w_sig_cert, &ctx->w_cert_first, &ctx->w_cert_n,
                      &ctx->w_msg, &ctx->w_msg_off, &ctx->w_msg_len, &ctx->w_flags, &ctx->w_slow_count,
                      &ctx->w_slow_list, &ctx->w_slow_slot, &ctx->w_slow_buf, &ctx->w_cert_ok, &ctx->w_stake_out,
                      &ctx->w_ok, &ctx->w_misc, &ctx->w_out, &ctx->w_pbuf, &ctx->w_pre,
                      &ctx->w_counts, &ctx->w_cursor, &ctx->w_perm, &ctx->w_io})
        b->release();
    ctx->h_io.release();
    for (auto& ev : ctx->prof_events) {
        (void)hipEventDestroy(ev.first);
        (void)hipEventDestroy(ev.second);
    }

    for (uint32_t* p : {ctx->d_btab, ctx->d_keys_raw, ctx->d_key_info, ctx->d_stake, ctx->d_key_tab})
        if (p) (void)hipFree(p);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

int nw_profile_enable(nw_ctx* ctx, int on) {
    if (!ctx) return NW_ERR_ARG;
    std::lock_guard<std::mutex> g(ctx->mu);
    ctx->prof_on = on != 0;
    return NW_OK;
}

int nw_profile_read(nw_ctx* ctx, double* verify_ms_total, uint64_t* verify_launches) {
    return nw_profile_read_sigs(ctx, verify_ms_total, verify_launches, nullptr);
}

int nw_profile_read_sigs(nw_ctx* ctx, double* verify_ms_total, uint64_t* verify_launches, uint64_t* verify_sigs) {
    if (!ctx) return NW_ERR_ARG;
    std::lock_guard<std::mutex> g(ctx->mu);
    NW_TRY(hipSetDevice(ctx->device), "hipSetDevice");
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

const char* nw_last_error(const nw_ctx* ctx) { return ctx ? ctx->last_error.c_str() : "null context"; }

size_t nw_committee_size(const nw_ctx* ctx) { return ctx ? ctx->nkeys : 0; }

int nw_key_window(const nw_ctx* ctx) { return ctx ? ctx->key_window : 0; }

int nw_base_window(void) { return B_WINDOW; }

int nw_committee_load(nw_ctx* ctx, const uint8_t (*pk)[32], const uint32_t* stake, size_t n, uint32_t* slot_out) {
    if (!ctx || (!pk && n)) return NW_ERR_ARG;
    std::lock_guard<std::mutex> g(ctx->mu);
    NW_TRY(hipSetDevice(ctx->device), "hipSetDevice");
    std::vector<uint32_t> slots(n);
    int rc = ensure_slots(ctx, pk, stake, n, slots.data());
    if (rc == NW_OK && slot_out) std::memcpy(slot_out, slots.data(), n * 4);
    return rc;
}

int nw_verify_strict_many(nw_ctx* ctx, const uint8_t* const* msg, const size_t* len, const uint8_t (*pk)[32],
                          const uint8_t (*sig)[64], size_t n, uint8_t* ok) {
    if (!ctx || !ok || (n && (!msg || !len || !pk || !sig))) return NW_ERR_ARG;
    if (n == 0) return NW_OK;
    std::lock_guard<std::mutex> g(ctx->mu);
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
    if (n == 0) return NW_OK;   // empty batch: the MSM is (-0)B = identity -> Ok
    std::lock_guard<std::mutex> g(ctx->mu);
    NW_TRY(hipSetDevice(ctx->device), "hipSetDevice");
    uint8_t verdict = 0;
    int rc = run_generic(ctx, msg, len, pk, sig, n, zseed, batch_index, 1, nullptr, &verdict);
    if (rc != NW_OK) return rc;
    return verdict ? NW_OK : NW_ERR_SIG;
}

int nw_verify_certs(nw_ctx* ctx, const nw_cert* certs, size_t ncerts, const uint8_t (*sig)[64],
                    const uint32_t* signer_slot, const uint8_t (*msg)[32], const uint8_t zseed[32], uint64_t cert_base,
                    uint8_t* cert_ok, uint8_t* sig_ok, uint64_t* accepted_stake) {
    if (!ctx || (ncerts && (!certs || !msg))) return NW_ERR_ARG;
    std::lock_guard<std::mutex> g(ctx->mu);
    NW_TRY(hipSetDevice(ctx->device), "hipSetDevice");
    size_t nsigs = 0;
    std::vector<uint32_t> first(ncerts), nv(ncerts);
    for (size_t c = 0; c < ncerts; ++c) {
        first[c] = certs[c].first_vote;
        nv[c] = certs[c].n_votes;
        const size_t end = (size_t)certs[c].first_vote + certs[c].n_votes;
        if (end > nsigs) nsigs = end;
    }
    if (nsigs && (!sig || !signer_slot)) return NW_ERR_ARG;
    for (size_t v = 0; v < nsigs; ++v)
        if (signer_slot[v] >= ctx->nkeys) {
            ctx->last_error = "signer slot out of range (load the committee first)";
            return NW_ERR_ARG;
        }
    if (ncerts == 0) return NW_OK;   // nothing to verify (nsigs is 0 too)
    // one staged H2D of every input and one D2H of every output (single-certificate latency)
    const size_t o_sig = 0, o_signer = align256(o_sig + nsigs * 64), o_first = align256(o_signer + nsigs * 4),
                 o_nv = align256(o_first + ncerts * 4), o_msg = align256(o_nv + ncerts * 4),
                 in_bytes = align256(o_msg + ncerts * 32);
    const size_t o_cok = 0, o_stake = align256(ncerts), o_ok = align256(o_stake + ncerts * 8),
                 out_bytes = align256(o_ok + nsigs);
    NW_TRY(ctx->w_io.ensure(in_bytes + out_bytes), "ws io");
    NW_TRY(ctx->h_io.ensure(in_bytes > out_bytes ? in_bytes : out_bytes), "pinned io");
    uint8_t* h = ctx->h_io.bytes();
    if (nsigs) {
        std::memcpy(h + o_sig, sig, nsigs * 64);
        std::memcpy(h + o_signer, signer_slot, nsigs * 4);
    }
    if (ncerts) {
        std::memcpy(h + o_first, first.data(), ncerts * 4);
        std::memcpy(h + o_nv, nv.data(), ncerts * 4);
        std::memcpy(h + o_msg, msg, ncerts * 32);
    }
    uint8_t* d_in = ctx->w_io.as<uint8_t>();
    uint8_t* d_out = d_in + in_bytes;
    hipStream_t st = ctx->stream;
    NW_TRY(hipMemcpyAsync(d_in, h, in_bytes, hipMemcpyHostToDevice, st), "H2D inputs");
    int rc = enqueue_certs(ctx, ncerts, reinterpret_cast<const uint32_t*>(d_in + o_first),
                           reinterpret_cast<const uint32_t*>(d_in + o_nv), nsigs, d_in + o_sig,
                           reinterpret_cast<const uint32_t*>(d_in + o_signer), 0, d_in + o_msg, nullptr, nullptr,
                           nullptr, zseed, cert_base, 1, d_out + o_cok, nullptr,
                           reinterpret_cast<uint64_t*>(d_out + o_stake), st);
    if (rc != NW_OK) return rc;
    if (sig_ok && nsigs)
        NW_TRY(launch_flags_to_ok((uint32_t)nsigs, ctx->w_flags.as<uint32_t>(), d_out + o_ok, st), "k_flags_to_ok");
    // the H2D above has completed in stream order before this copy overwrites the staging buffer
    NW_TRY(hipMemcpyAsync(h, d_out, out_bytes, hipMemcpyDeviceToHost, st), "D2H outputs");
    NW_TRY(hipStreamSynchronize(st), "sync");
    if (sig_ok && nsigs) std::memcpy(sig_ok, h + o_ok, nsigs);
    if (cert_ok && ncerts) std::memcpy(cert_ok, h + o_cok, ncerts);
    if (accepted_stake && ncerts) std::memcpy(accepted_stake, h + o_stake, ncerts * 8);
    return NW_OK;
}

int nw_verify_batches(nw_ctx* ctx, size_t nb, const uint32_t* first, const uint32_t* nvotes,
                      const uint8_t* const* msg, const size_t* len, const uint32_t* signer_slot,
                      const uint8_t (*sig)[64], const uint8_t zseed[32], uint64_t batch_base, uint8_t* batch_ok,
                      uint8_t* sig_ok) {
    if (!ctx || (nb && (!first || !nvotes))) return NW_ERR_ARG;
    std::lock_guard<std::mutex> g(ctx->mu);
    NW_TRY(hipSetDevice(ctx->device), "hipSetDevice");
    size_t nsigs = 0;
    for (size_t b = 0; b < nb; ++b) {
        const size_t end = (size_t)first[b] + nvotes[b];
        if (end > nsigs) nsigs = end;
    }
    if (nsigs && (!sig || !signer_slot || !msg || !len)) return NW_ERR_ARG;
    for (size_t v = 0; v < nsigs; ++v)
        if (signer_slot[v] >= ctx->nkeys) {
            ctx->last_error = "signer slot out of range (load the keys first)";
            return NW_ERR_ARG;
        }
    hipStream_t st = ctx->stream;
    int rc = upload_messages(ctx, msg, len, nsigs);
    if (rc != NW_OK) return rc;
    NW_TRY(ctx->w_sig.ensure(nsigs * 64 + 64), "ws sig");
    NW_TRY(ctx->w_signer.ensure(nsigs * 4 + 4), "ws signer");
    NW_TRY(ctx->w_cert_first.ensure(nb * 4 + 4), "ws first");
    NW_TRY(ctx->w_cert_n.ensure(nb * 4 + 4), "ws n");
    NW_TRY(ctx->w_cert_ok.ensure(nb + 16), "ws batch_ok");
    NW_TRY(ctx->w_ok.ensure(nsigs + 16), "ws ok");
    if (nsigs) {
        NW_TRY(hipMemcpyAsync(ctx->w_sig.p, sig, nsigs * 64, hipMemcpyHostToDevice, st), "H2D sig");
        NW_TRY(hipMemcpyAsync(ctx->w_signer.p, signer_slot, nsigs * 4, hipMemcpyHostToDevice, st), "H2D signer");
    }
    if (nb) {
        NW_TRY(hipMemcpyAsync(ctx->w_cert_first.p, first, nb * 4, hipMemcpyHostToDevice, st), "H2D first");
        NW_TRY(hipMemcpyAsync(ctx->w_cert_n.p, nvotes, nb * 4, hipMemcpyHostToDevice, st), "H2D n");
    }
    rc = enqueue_certs(ctx, nb, ctx->w_cert_first.as<uint32_t>(), ctx->w_cert_n.as<uint32_t>(), nsigs,
                       ctx->w_sig.as<uint8_t>(), ctx->w_signer.as<uint32_t>(), 1, nullptr, ctx->w_msg.as<uint8_t>(),
                       ctx->w_msg_off.as<uint64_t>(), ctx->w_msg_len.as<uint64_t>(), zseed, batch_base, 1,
                       ctx->w_cert_ok.as<uint8_t>(), nullptr, nullptr, st);
    if (rc != NW_OK) return rc;
    if (sig_ok && nsigs) {
        NW_TRY(launch_flags_to_ok((uint32_t)nsigs, ctx->w_flags.as<uint32_t>(), ctx->w_ok.as<uint8_t>(), st),
               "k_flags_to_ok");
        NW_TRY(hipMemcpyAsync(sig_ok, ctx->w_ok.p, nsigs, hipMemcpyDeviceToHost, st), "D2H sig_ok");
    }
    if (batch_ok && nb) NW_TRY(hipMemcpyAsync(batch_ok, ctx->w_cert_ok.p, nb, hipMemcpyDeviceToHost, st), "D2H");
    NW_TRY(hipStreamSynchronize(st), "sync");
    return NW_OK;
}

int nw_verify_certs_dev(nw_ctx* ctx, size_t ncerts, const uint32_t* d_cert_first, const uint32_t* d_cert_nvotes,
                        size_t nsigs, const uint8_t* d_sig64, const uint32_t* d_signer_slot, const uint8_t* d_msg32,
                        const uint8_t zseed[32], uint64_t cert_base, uint8_t* d_cert_ok, uint32_t* d_sig_flags,
                        uint64_t* d_accepted_stake, void* stream) {
    if (!ctx) return NW_ERR_ARG;
    std::lock_guard<std::mutex> g(ctx->mu);
    NW_TRY(hipSetDevice(ctx->device), "hipSetDevice");
    return enqueue_certs(ctx, ncerts, d_cert_first, d_cert_nvotes, nsigs, d_sig64, d_signer_slot, 0, d_msg32, nullptr,
                         nullptr, nullptr, zseed, cert_base, 1, d_cert_ok, d_sig_flags, d_accepted_stake,
                         reinterpret_cast<hipStream_t>(stream));
}

int nw_sha512_many_dev(nw_ctx* ctx, const uint8_t* d_base, const uint64_t* d_off, const uint64_t* d_len, size_t n,
                       uint8_t* d_out64, void* stream) {
    if (!ctx) return NW_ERR_ARG;
    std::lock_guard<std::mutex> g(ctx->mu);
    NW_TRY(hipSetDevice(ctx->device), "hipSetDevice");
    NW_TRY(launch_sha512_many((uint32_t)n, d_base, d_off, d_len, d_out64, reinterpret_cast<hipStream_t>(stream)),
           "k_sha512_many");
    return NW_OK;
}

int nw_sha512_many(nw_ctx* ctx, const uint8_t* base, const uint64_t* off, const uint64_t* len, size_t n,
                   uint8_t (*out)[64]) {
    if (!ctx || (n && (!off || !len || !out))) return NW_ERR_ARG;
    if (n == 0) return NW_OK;
    std::lock_guard<std::mutex> g(ctx->mu);
    NW_TRY(hipSetDevice(ctx->device), "hipSetDevice");
    // upload only the referenced span
    uint64_t lo = UINT64_MAX, hi = 0;
    for (size_t i = 0; i < n; ++i) {
        if (off[i] < lo) lo = off[i];
        if (off[i] + len[i] > hi) hi = off[i] + len[i];
    }
    if (hi < lo) hi = lo;
    std::vector<uint64_t> roff(n);
    for (size_t i = 0; i < n; ++i) roff[i] = off[i] - lo;
    const size_t span = (size_t)(hi - lo);
    hipStream_t st = ctx->stream;
    NW_TRY(ctx->w_msg.ensure(span + 16), "ws msg");
    NW_TRY(ctx->w_msg_off.ensure(n * 8), "ws off");
    NW_TRY(ctx->w_msg_len.ensure(n * 8), "ws len");
    NW_TRY(ctx->w_out.ensure(n * 64), "ws out");
    if (span) NW_TRY(hipMemcpyAsync(ctx->w_msg.p, base + lo, span, hipMemcpyHostToDevice, st), "H2D data");
    NW_TRY(hipMemcpyAsync(ctx->w_msg_off.p, roff.data(), n * 8, hipMemcpyHostToDevice, st), "H2D off");
    NW_TRY(hipMemcpyAsync(ctx->w_msg_len.p, len, n * 8, hipMemcpyHostToDevice, st), "H2D len");
    NW_TRY(launch_sha512_many((uint32_t)n, ctx->w_msg.as<uint8_t>(), ctx->w_msg_off.as<uint64_t>(),
                              ctx->w_msg_len.as<uint64_t>(), ctx->w_out.as<uint8_t>(), st),
           "k_sha512_many");
    NW_TRY(hipMemcpyAsync(out, ctx->w_out.p, n * 64, hipMemcpyDeviceToHost, st), "D2H digests");
    NW_TRY(hipStreamSynchronize(st), "sync");
    return NW_OK;
}

int nw_sha512(nw_ctx* ctx, const uint8_t* data, size_t len, uint8_t out[64]) {
    const uint64_t off = 0, ln = len;
    static const uint8_t empty[1] = {0};
    return nw_sha512_many(ctx, data ? data : empty, &off, &ln, 1, reinterpret_cast<uint8_t(*)[64]>(out));
}

int nw_sign_many_dev(nw_ctx* ctx, const uint8_t* d_seed32, const uint8_t* d_msgs, size_t msg_len, size_t n,
                     uint8_t* d_pk32, uint8_t* d_sig64, void* stream) {
    if (!ctx || (msg_len != 8 && msg_len != 32)) return NW_ERR_ARG;
    std::lock_guard<std::mutex> g(ctx->mu);
    NW_TRY(hipSetDevice(ctx->device), "hipSetDevice");
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
    std::lock_guard<std::mutex> g(ctx->mu);
    NW_TRY(hipSetDevice(ctx->device), "hipSetDevice");
    hipStream_t st = ctx->stream;
    NW_TRY(ctx->w_misc.ensure(n * 32 + n * msg_len + 16), "ws misc");
    NW_TRY(ctx->w_out.ensure(n * 96 + 16), "ws out");
    uint8_t* d_seed = ctx->w_misc.as<uint8_t>();
    uint8_t* d_msg = d_seed + n * 32;
    uint8_t* d_pk = ctx->w_out.as<uint8_t>();
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
    return NW_OK;
}

}  // extern "C"
