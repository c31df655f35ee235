// Native ingestion of the primary's certificate traffic and the whole of
// Certificate::verify over many certificates, host side in C++.
//
//   wire:   bincode 1.3 (fixint, little endian, trailing bytes allowed: bincode::deserialize as called
//           at primary/src/primary.rs:236) PrimaryMessage frames; variant 2 = Certificate
//           (primary/src/primary.rs:33-38, derives at primary/src/messages.rs:13-21,105-111,168-172).
//           PublicKey is its base64 string (crypto/src/lib.rs:68-112); Digest 32 raw bytes;
//           Signature part1 || part2 = 64 raw bytes.
//   checks: Certificate::verify (primary/src/messages.rs:189-215) -> Header::verify (:48-67), in the
//           reference's order, each failure reported as the DagError kind it returns
//           (primary/src/error.rs:24-58).
//
// Decoding writes a struct-of-arrays batch (signer committee index, 64-byte signature per vote;
// header / certificate digest preimages per certificate) that feeds the GPU in three submissions
// with no per-vote objects: one nw_sha512_many (header ids and certificate digests), one
// nw_verify_strict_many (header signatures), one nw_verify_certs (every vote of every certificate
// that reached the batch step).  Nothing here computes a digest or a verdict on the CPU.
#include <algorithm>
#include <array>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/nwcrypto.h"

namespace {

using Key = std::array<uint8_t, 32>;

struct KeyHash {
    size_t operator()(const Key& k) const {
        uint64_t h;
        std::memcpy(&h, k.data(), 8);   // keys are curve points: uniformly distributed bytes
        return (size_t)(h ^ (h >> 29));
    }
};

// base64 0.13 STANDARD decoding (crypto/src/lib.rs:73), restated from the published crate's
// decode_suffix (not vendored here: parity unpinned, tests/golden/README.md): alphabet A-Z a-z 0-9
// + /; '=' is padding only in the final quantum, only at positions 2 and 3 of a quad (counted
// from the start of the string) and with nothing but '=' after it; padding is NOT required to
// complete the quad (46 symbols + one '=' decodes) and may be absent; a final quantum of one
// symbol is InvalidLength; non-zero trailing bits of the last symbol are InvalidLastSymbol.
int b64val(uint8_t c) {
    if (c >= 'A' && c <= 'Z') return c - 'A';
    if (c >= 'a' && c <= 'z') return c - 'a' + 26;
    if (c >= '0' && c <= '9') return c - '0' + 52;
    if (c == '+') return 62;
    if (c == '/') return 63;
    return -1;
}

bool b64_decode(const uint8_t* s, size_t n, std::vector<uint8_t>& out) {
    size_t m = 0;                 // symbols before the first '='
    while (m < n && s[m] != '=') ++m;
    for (size_t i = m; i < n; ++i)   // padding: only '=', each at quad position 2 or 3
        if (s[i] != '=' || i % 4 < 2) return false;
    if (n - m > 2) return false;
    if (m % 4 == 1) return false;
    out.clear();
    out.reserve(m * 3 / 4);
    uint32_t acc = 0;
    int bits = 0;
    for (size_t i = 0; i < m; ++i) {
        const int v = b64val(s[i]);
        if (v < 0) return false;
        acc = (acc << 6) | (uint32_t)v;
        bits += 6;
        if (bits >= 8) {
            bits -= 8;
            out.push_back((uint8_t)(acc >> bits));
            acc &= (1u << bits) - 1u;
        }
    }
    return acc == 0;   // leftover bits of the last symbol must be zero
}

struct Reader {
    const uint8_t* p;
    size_t n, at = 0;
    bool ok = true;
    bool take(size_t k, const uint8_t** out) {
        if (!ok || k > n - at) return ok = false;
        *out = p + at;
        at += k;
        return true;
    }
    uint64_t u64() {
        const uint8_t* b;
        if (!take(8, &b)) return 0;
        uint64_t v;
        std::memcpy(&v, b, 8);
        return v;
    }
    uint32_t u32() {
        const uint8_t* b;
        if (!take(4, &b)) return 0;
        uint32_t v;
        std::memcpy(&v, b, 4);
        return v;
    }
    // PublicKey: String (u64 length + UTF-8) holding base64; the first 32 decoded bytes
    // (crypto/src/lib.rs:72-79).  A decoded length < 32 panics in the reference (bytes[..32]);
    // here it is a serialization error.
    bool public_key(Key& k, std::vector<uint8_t>& scratch) {
        const uint64_t len = u64();
        const uint8_t* s;
        if (!ok || len > n - at || !take((size_t)len, &s)) return ok = false;
        if (!b64_decode(s, (size_t)len, scratch) || scratch.size() < 32) return ok = false;
        std::memcpy(k.data(), scratch.data(), 32);
        return true;
    }
};

}  // namespace

struct nw_cert_batch {
    struct Cert {
        int32_t status = NW_DAG_PENDING;
        int32_t header_error = NW_DAG_OK;   // Header::verify host checks after the id check
        int32_t quorum_error = NW_DAG_OK;   // Certificate::verify quorum checks
        uint64_t round = 0;
        Key author{};
        uint8_t id[32] = {0};
        uint8_t sig[64] = {0};
        std::vector<uint8_t> header_pre;
        uint8_t cert_pre[72] = {0};
        uint32_t first_vote = 0, n_votes = 0;
    };
    std::vector<Cert> certs;
    std::vector<uint8_t> vote_pk;      // [V][32]
    std::vector<uint8_t> vote_sig;     // [V][64]
    std::vector<uint32_t> vote_member; // committee index of the vote's author (valid when quorum passed)
    std::vector<Key> names;            // committee names (nw_committee_load order)
    std::vector<uint32_t> stakes;
};

namespace {

// Header (primary/src/messages.rs:13-21) + its digest preimage (:70-84): author || round ||
// (digest || worker_id)* || parents*, with the BTreeMap / BTreeSet semantics of the deserialized
// containers (sorted, duplicate payload keys keep the last value, duplicate parents collapse).
bool read_header(Reader& r, nw_cert_batch::Cert& c, std::vector<uint32_t>& workers, std::vector<uint8_t>& scratch) {
    if (!r.public_key(c.author, scratch)) return false;
    c.round = r.u64();
    const uint64_t np = r.u64();
    if (!r.ok || np > (r.n - r.at) / 36) return false;
    std::vector<std::pair<Key, uint32_t>> payload;
    payload.reserve((size_t)np);
    bool sorted = true;
    for (uint64_t i = 0; i < np; ++i) {
        const uint8_t* d;
        if (!r.take(32, &d)) return false;
        Key k;
        std::memcpy(k.data(), d, 32);
        const uint32_t w = r.u32();
        if (!payload.empty() && !(payload.back().first < k)) sorted = false;
        payload.emplace_back(k, w);
    }
    if (!sorted) {   // BTreeMap: last insert wins per key, iteration in key order
        std::stable_sort(payload.begin(), payload.end(),
                         [](const std::pair<Key, uint32_t>& a, const std::pair<Key, uint32_t>& b) { return a.first < b.first; });
        std::vector<std::pair<Key, uint32_t>> u;
        for (auto& e : payload) {
            if (!u.empty() && u.back().first == e.first) u.back().second = e.second;
            else u.push_back(e);
        }
        payload.swap(u);
    }
    const uint64_t nparents = r.u64();
    if (!r.ok || nparents > (r.n - r.at) / 32) return false;
    const uint8_t* pp;
    if (!r.take((size_t)nparents * 32, &pp)) return false;
    std::vector<Key> parents((size_t)nparents);
    for (size_t i = 0; i < parents.size(); ++i) std::memcpy(parents[i].data(), pp + 32 * i, 32);
    if (!std::is_sorted(parents.begin(), parents.end()) ||
        std::adjacent_find(parents.begin(), parents.end()) != parents.end()) {
        std::sort(parents.begin(), parents.end());
        parents.erase(std::unique(parents.begin(), parents.end()), parents.end());
    }
    const uint8_t *id, *sig;
    if (!r.take(32, &id) || !r.take(64, &sig)) return false;
    std::memcpy(c.id, id, 32);
    std::memcpy(c.sig, sig, 64);
    c.header_pre.resize(40 + 36 * payload.size() + 32 * parents.size());
    uint8_t* o = c.header_pre.data();
    std::memcpy(o, c.author.data(), 32);
    std::memcpy(o + 32, &c.round, 8);
    o += 40;
    workers.clear();
    for (auto& e : payload) {
        std::memcpy(o, e.first.data(), 32);
        std::memcpy(o + 32, &e.second, 4);
        o += 36;
        workers.push_back(e.second);
    }
    for (auto& p : parents) {
        std::memcpy(o, p.data(), 32);
        o += 32;
    }
    return true;
}

}  // namespace

extern "C" {

int nw_cert_batch_decode(const nw_committee* cm, const uint8_t* const* frame, const size_t* len, size_t n,
                         nw_cert_batch** out) {
    if (!out || !cm || (cm->n && (!cm->name || !cm->stake)) || (n && (!frame || !len))) return NW_ERR_ARG;
    *out = nullptr;
    auto* b = new (std::nothrow) nw_cert_batch;
    if (!b) return NW_ERR_NOMEM;
    std::unordered_map<Key, uint32_t, KeyHash> member;   // Committee.authorities (config/src/lib.rs:161-177)
    member.reserve(cm->n * 2);
    b->names.resize(cm->n);
    b->stakes.assign(cm->stake, cm->stake + cm->n);
    uint64_t total = 0;
    for (size_t i = 0; i < cm->n; ++i) {
        std::memcpy(b->names[i].data(), cm->name[i], 32);
        member.emplace(b->names[i], (uint32_t)i);
        total += cm->stake[i];
    }
    const uint64_t quorum = 2 * total / 3 + 1;   // Committee::quorum_threshold (config/src/lib.rs:189-194)
    auto stake_of = [&](const Key& k, uint32_t* idx) -> uint64_t {
        auto it = member.find(k);
        if (it == member.end()) return 0;
        if (idx) *idx = it->second;
        return cm->stake[it->second];
    };
    auto has_worker = [&](uint32_t a, uint32_t w) {   // Committee::worker (config/src/lib.rs:229-240)
        if (!cm->worker_first || !cm->worker_id) return false;
        for (uint32_t k = cm->worker_first[a]; k < cm->worker_first[a + 1]; ++k)
            if (cm->worker_id[k] == w) return true;
        return false;
    };
    b->certs.resize(n);
    std::vector<uint8_t> scratch;
    std::vector<uint32_t> workers;
    std::vector<uint32_t> used;
    for (size_t i = 0; i < n; ++i) {
        auto& c = b->certs[i];
        if (!frame[i] && len[i]) {
            delete b;
            return NW_ERR_ARG;
        }
        Reader r{frame[i], len[i]};
        const uint32_t tag = r.u32();
        if (!r.ok || tag > 3) {
            c.status = NW_DAG_SERIALIZATION;
            continue;
        }
        if (tag != 2) {
            c.status = NW_DAG_NOT_CERTIFICATE;
            continue;
        }
        if (!read_header(r, c, workers, scratch)) {
            c.status = NW_DAG_SERIALIZATION;
            continue;
        }
        const uint64_t nv = r.u64();
        if (!r.ok || nv > (r.n - r.at) / 72) {   // each vote takes >= 8 + 64 bytes
            c.status = NW_DAG_SERIALIZATION;
            continue;
        }
        const size_t v0 = b->vote_sig.size() / 64;
        bool good = true;
        for (uint64_t v = 0; v < nv && good; ++v) {
            Key k;
            const uint8_t* s;
            good = r.public_key(k, scratch) && r.take(64, &s);
            if (good) {
                b->vote_pk.insert(b->vote_pk.end(), k.begin(), k.end());
                b->vote_sig.insert(b->vote_sig.end(), s, s + 64);
            }
        }
        if (!good) {   // drop this certificate's partial votes
            b->vote_pk.resize(v0 * 32);
            b->vote_sig.resize(v0 * 64);
            c.status = NW_DAG_SERIALIZATION;
            continue;
        }
        // bincode::deserialize allows trailing bytes: nothing to check past the votes.
        c.first_vote = (uint32_t)v0;
        c.n_votes = (uint32_t)nv;
        b->vote_member.resize(v0 + nv, 0);
        // Certificate digest preimage (:226-234): header.id || round || origin.
        std::memcpy(c.cert_pre, c.id, 32);
        std::memcpy(c.cert_pre + 32, &c.round, 8);
        std::memcpy(c.cert_pre + 40, c.author.data(), 32);
        // Genesis (:191-193 with PartialEq at :249-256): same id, round and origin as a genesis
        // certificate, i.e. id = Digest::default(), round 0, origin a committee member.
        static const uint8_t zero[32] = {0};
        uint32_t aidx = 0;
        const uint64_t astake = stake_of(c.author, &aidx);
        if (c.round == 0 && std::memcmp(c.id, zero, 32) == 0 && member.count(c.author)) {
            c.status = NW_DAG_OK;
            continue;
        }
        // Header::verify after the id check: author stake, then every payload worker id.
        if (astake == 0) {
            c.header_error = NW_DAG_UNKNOWN_AUTHORITY;
        } else {
            for (uint32_t w : workers)
                if (!has_worker(aidx, w)) {
                    c.header_error = NW_DAG_MALFORMED_HEADER;
                    break;
                }
        }
        // Quorum (:199-211): reuse, unknown authority, then the 2f+1 threshold.
        uint64_t weight = 0;
        used.clear();
        for (uint32_t v = 0; v < nv; ++v) {
            Key k;
            std::memcpy(k.data(), &b->vote_pk[(v0 + v) * 32], 32);
            uint32_t idx = 0;
            const uint64_t st = stake_of(k, &idx);
            if (st && std::find(used.begin(), used.end(), idx) != used.end()) {
                c.quorum_error = NW_DAG_AUTHORITY_REUSE;
                break;
            }
            if (st == 0) {   // only known names enter `used`, so an unknown name fails here first
                c.quorum_error = NW_DAG_UNKNOWN_AUTHORITY;
                break;
            }
            used.push_back(idx);
            b->vote_member[v0 + v] = idx;
            weight += st;
        }
        if (c.quorum_error == NW_DAG_OK && weight < quorum) c.quorum_error = NW_DAG_REQUIRES_QUORUM;
    }
    *out = b;
    return NW_OK;
}

void nw_cert_batch_free(nw_cert_batch* b) { delete b; }

size_t nw_cert_batch_size(const nw_cert_batch* b) { return b ? b->certs.size() : 0; }

int nw_cert_batch_view(const nw_cert_batch* b, size_t i, nw_cert_view* out) {
    if (!b || !out || i >= b->certs.size()) return NW_ERR_ARG;
    const auto& c = b->certs[i];
    out->status = c.status;
    out->header_error = c.header_error;
    out->quorum_error = c.quorum_error;
    out->round = c.round;
    out->author = c.author.data();
    out->header_id = c.id;
    out->header_sig = c.sig;
    out->header_preimage = c.header_pre.data();
    out->header_preimage_len = c.header_pre.size();
    out->cert_preimage = c.cert_pre;
    out->first_vote = c.first_vote;
    out->n_votes = c.n_votes;
    out->vote_keys = b->vote_pk.data() + (size_t)c.first_vote * 32;
    out->vote_sigs = b->vote_sig.data() + (size_t)c.first_vote * 64;
    return NW_OK;
}

int nw_cert_batch_verify(nw_ctx* ctx, const nw_cert_batch* b, const uint8_t zseed[32], uint64_t cert_base,
                         int32_t* verdict) {
    if (!ctx || !b || !zseed || (!verdict && !b->certs.empty())) return NW_ERR_ARG;
    const size_t n = b->certs.size();
    std::vector<size_t> todo;
    for (size_t i = 0; i < n; ++i) {
        verdict[i] = b->certs[i].status;
        if (b->certs[i].status == NW_DAG_PENDING) todo.push_back(i);
    }
    if (todo.empty()) return NW_OK;
    // 1. header ids and certificate digests: one SHA-512 submission
    std::vector<uint64_t> off, len;
    std::vector<uint8_t> buf;
    for (size_t i : todo) {
        off.push_back(buf.size());
        len.push_back(b->certs[i].header_pre.size());
        buf.insert(buf.end(), b->certs[i].header_pre.begin(), b->certs[i].header_pre.end());
    }
    for (size_t i : todo) {
        off.push_back(buf.size());
        len.push_back(72);
        buf.insert(buf.end(), b->certs[i].cert_pre, b->certs[i].cert_pre + 72);
    }
    std::vector<uint8_t> dig(off.size() * 64);
    int rc = nw_sha512_many(ctx, buf.data(), off.data(), len.data(), off.size(), reinterpret_cast<uint8_t(*)[64]>(dig.data()));
    if (rc != NW_OK) return rc;
    // Committee keys go to the context's key cache once (nw_committee_load deduplicates), so the
    // header signatures and the vote batches below take the cached comb path.
    std::vector<uint32_t> slot(b->names.size());
    rc = nw_committee_load(ctx, reinterpret_cast<const uint8_t(*)[32]>(b->names.data()), b->stakes.data(),
                           b->names.size(), slot.data());
    if (rc != NW_OK) return rc;
    // 2. Header::verify: id, then the host checks, then the strict signature (one submission)
    std::vector<size_t> live;
    for (size_t k = 0; k < todo.size(); ++k) {
        const auto& c = b->certs[todo[k]];
        if (std::memcmp(&dig[k * 64], c.id, 32) != 0) verdict[todo[k]] = NW_DAG_INVALID_HEADER_ID;
        else if (c.header_error != NW_DAG_OK) verdict[todo[k]] = c.header_error;
        else live.push_back(k);
    }
    if (!live.empty()) {
        std::vector<const uint8_t*> msg;
        std::vector<size_t> mlen;
        std::vector<uint8_t> pk, sg;
        for (size_t k : live) {
            const auto& c = b->certs[todo[k]];
            msg.push_back(c.id);
            mlen.push_back(32);
            pk.insert(pk.end(), c.author.begin(), c.author.end());
            sg.insert(sg.end(), c.sig, c.sig + 64);
        }
        std::vector<uint8_t> ok(live.size());
        rc = nw_verify_strict_many(ctx, msg.data(), mlen.data(), reinterpret_cast<const uint8_t(*)[32]>(pk.data()),
                                   reinterpret_cast<const uint8_t(*)[64]>(sg.data()), live.size(), ok.data());
        if (rc != NW_OK) return rc;
        std::vector<size_t> nxt;
        for (size_t j = 0; j < live.size(); ++j) {
            const auto& c = b->certs[todo[live[j]]];
            if (!ok[j]) verdict[todo[live[j]]] = NW_DAG_INVALID_SIGNATURE;
            else if (c.quorum_error != NW_DAG_OK) verdict[todo[live[j]]] = c.quorum_error;
            else nxt.push_back(live[j]);
        }
        live.swap(nxt);
    }
    if (live.empty()) return NW_OK;
    // 3. Signature::verify_batch of every remaining certificate: one submission.
    std::vector<nw_cert> certs;
    std::vector<uint32_t> signer;
    std::vector<uint8_t> sigs, msgs;
    for (size_t k : live) {
        const auto& c = b->certs[todo[k]];
        certs.push_back({(uint32_t)signer.size(), c.n_votes});
        for (uint32_t v = 0; v < c.n_votes; ++v) signer.push_back(slot[b->vote_member[c.first_vote + v]]);
        sigs.insert(sigs.end(), b->vote_sig.begin() + (size_t)c.first_vote * 64,
                    b->vote_sig.begin() + ((size_t)c.first_vote + c.n_votes) * 64);
        msgs.insert(msgs.end(), &dig[(todo.size() + k) * 64], &dig[(todo.size() + k) * 64] + 32);
    }
    std::vector<uint8_t> cert_ok(certs.size());
    rc = nw_verify_certs(ctx, certs.data(), certs.size(), reinterpret_cast<const uint8_t(*)[64]>(sigs.data()),
                         signer.data(), reinterpret_cast<const uint8_t(*)[32]>(msgs.data()), zseed, cert_base,
                         cert_ok.data(), nullptr, nullptr);
    if (rc != NW_OK) return rc;
    for (size_t j = 0; j < live.size(); ++j)
        verdict[todo[live[j]]] = cert_ok[j] ? NW_DAG_OK : NW_DAG_INVALID_SIGNATURE;
    return NW_OK;
}

int nw_certificates_verify(nw_ctx* ctx, const nw_committee* cm, const uint8_t* const* frame, const size_t* len,
                           size_t n, const uint8_t zseed[32], uint64_t cert_base, int32_t* verdict) {
    if (!ctx) return NW_ERR_ARG;
    nw_cert_batch* b = nullptr;
    int rc = nw_cert_batch_decode(cm, frame, len, n, &b);
    if (rc != NW_OK) return rc;
    rc = nw_cert_batch_verify(ctx, b, zseed, cert_base, verdict);
    nw_cert_batch_free(b);
    return rc;
}

}  // extern "C"
