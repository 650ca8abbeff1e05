// Mash sketch databases (.msh) read natively: the S1 row of the screen stage.
//
// `mash screen` re-reads its sketch database on every call (scripts/mash.sh:14; the three
// DBs of run_hymet_cami.sh:85-97 are read once each per run), so the .msh parse is on the
// timed path.  A .msh file is one Cap'n Proto message in the standard unpacked framing
// (segment table, then segments), holding Mash's MinHash struct (restated in
// hymet_amd/msh.py; Mash is third-party and not in the image).  This reader maps the file,
// walks the pointers itself -- near, single-far and double-far pointers, any segment count,
// bounds-checked -- and gathers every reference's hash list into one CSR array on host
// threads, widening 32-bit hashes (k <= 16) to uint64 and sorting any list that is not
// already ascending.  No Cap'n Proto library is needed.
//
// Which pointer is the reference list: the schema keeps the pre-2.0 list as
// `referenceListOld` (pointer 0) and the current one beside the locus list (pointers 1/2).
// The current list is the one whose elements are Reference structs (they carry pointers;
// Locus elements carry none); it is used when it holds any reference, else the old list,
// as Mash's loader does.
#include "common.hpp"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <memory>
#include <cstring>
#include <thread>
#include <vector>

struct hymet_msh {
    const uint8_t *map = nullptr;
    size_t map_len = 0;
    std::vector<std::pair<int64_t, int64_t>> seg;  // (byte offset in file, words)
    hymet_msh_info info{};
    struct Ref {
        int64_t name_off, name_len, comment_off, comment_len;  // byte ranges in the file
        int64_t hash_off, n_hash;                              // byte offset of the list, entries
        int64_t length;
    };
    std::vector<Ref> refs;
    int64_t alphabet_off = 0, alphabet_len = 0;
};

namespace {

struct Ptr {  // a resolved pointer: target segment / word and the describing pointer word
    int seg = -1;
    int64_t word = 0;
    uint64_t desc = 0;
    bool null = true;
};

struct Reader {
    hymet_msh *m;
    std::string err;

    bool fail(const char *msg) {
        if (err.empty()) err = msg;
        return false;
    }
    bool word_at(int seg, int64_t w, uint64_t *out) {
        if (seg < 0 || seg >= (int)m->seg.size() || w < 0 || w >= m->seg[seg].second) return fail("pointer out of bounds");
        memcpy(out, m->map + m->seg[seg].first + 8 * w, 8);
        return true;
    }
    // the pointer stored at (seg, w)
    bool resolve(int seg, int64_t w, Ptr *out) {
        uint64_t p;
        if (!word_at(seg, w, &p)) return false;
        *out = Ptr{};
        if (p == 0) return true;
        const int kind = (int)(p & 3);
        if (kind == 2) {  // far pointer: landing pad in segment p >> 32
            const bool dbl = (p >> 2) & 1;
            const int tseg = (int)(p >> 32);
            const int64_t land = (int64_t)((p >> 3) & ((1ull << 29) - 1));
            if (!dbl) {
                // single-far: the landing pad is an ordinary struct / list pointer in the
                // target segment; a far or capability pad there is malformed (and a far pad
                // could loop), so decode it here without recursing
                uint64_t pad;
                if (!word_at(tseg, land, &pad)) return false;
                if (pad == 0) return true;
                if ((pad & 3) >= 2) return fail("far pointer landing pad is not a struct or list pointer");
                int64_t poff = (int64_t)((pad >> 2) & ((1ull << 30) - 1));
                if (poff & (1ll << 29)) poff -= 1ll << 30;
                out->seg = tseg;
                out->word = land + 1 + poff;
                out->desc = pad;
                out->null = false;
                return true;
            }
            uint64_t pad0, pad1;
            if (!word_at(tseg, land, &pad0) || !word_at(tseg, land + 1, &pad1)) return false;
            if ((pad0 & 3) != 2 || ((pad0 >> 2) & 1)) return fail("bad double-far landing pad");
            out->seg = (int)(pad0 >> 32);
            out->word = (int64_t)((pad0 >> 3) & ((1ull << 29) - 1));
            out->desc = pad1;
            out->null = false;
            if (out->seg < 0 || out->seg >= (int)m->seg.size()) return fail("far pointer segment out of range");
            return true;
        }
        if (kind == 3) return fail("capability pointer in a .msh message");
        int64_t off = (int64_t)((p >> 2) & ((1ull << 30) - 1));
        if (off & (1ll << 29)) off -= 1ll << 30;
        out->seg = seg;
        out->word = w + 1 + off;
        out->desc = p;
        out->null = false;
        return true;
    }
};

struct Struct {
    int seg = -1;
    int64_t word = 0;
    int dwords = 0, nptrs = 0;
    bool null = true;
};

bool as_struct(Reader &r, const Ptr &p, Struct *s) {
    *s = Struct{};
    if (p.null) return true;
    if ((p.desc & 3) != 0) return r.fail("expected a struct pointer");
    s->seg = p.seg;
    s->word = p.word;
    s->dwords = (int)((p.desc >> 32) & 0xFFFF);
    s->nptrs = (int)(p.desc >> 48);
    s->null = false;
    if (s->word < 0 || s->word + s->dwords + s->nptrs > r.m->seg[s->seg].second) return r.fail("struct out of bounds");
    return true;
}

bool struct_ptr(Reader &r, const Struct &s, int i, Ptr *out) {
    *out = Ptr{};
    if (s.null || i >= s.nptrs) return true;  // field absent in an older writer: default (null)
    return r.resolve(s.seg, s.word + s.dwords + i, out);
}

uint64_t data_u64(Reader &r, const Struct &s, int byte_off, int bytes) {  // little-endian, 0 past the data section
    if (s.null || byte_off + bytes > 8 * s.dwords) return 0;
    uint64_t v = 0;
    memcpy(&v, r.m->map + r.m->seg[s.seg].first + 8 * s.word + byte_off, (size_t)bytes);
    return v;
}

bool data_bit(Reader &r, const Struct &s, int bit) {
    if (s.null || bit >= 64 * s.dwords) return false;
    const uint8_t b = r.m->map[r.m->seg[s.seg].first + 8 * s.word + bit / 8];
    return (b >> (bit % 8)) & 1;
}

// a primitive list: byte offset of its first element in the file and its element count
bool prim_list(Reader &r, const Ptr &p, int want_code, int64_t *byte_off, int64_t *count) {
    *byte_off = 0;
    *count = 0;
    if (p.null) return true;
    if ((p.desc & 3) != 1) return r.fail("expected a list pointer");
    const int code = (int)((p.desc >> 32) & 7);
    const int64_t n = (int64_t)(p.desc >> 35);
    if (code != want_code) return r.fail("unexpected list element size");
    static const int bits[8] = {0, 1, 8, 16, 32, 64, 64, 0};
    const int64_t words = (n * bits[code] + 63) / 64;
    if (p.word < 0 || p.word + words > r.m->seg[p.seg].second) return r.fail("list out of bounds");
    *byte_off = r.m->seg[p.seg].first + 8 * p.word;
    *count = n;
    return true;
}

// Text: bytes with a trailing NUL (dropped)
bool text(Reader &r, const Ptr &p, int64_t *off, int64_t *len) {
    int64_t o, n;
    if (!prim_list(r, p, 2, &o, &n)) return false;
    if (n > 0 && r.m->map[o + n - 1] == 0) n--;
    *off = o;
    *len = n;
    return true;
}

// composite list: (segment, first element word, count, element data words, element pointers)
bool struct_list(Reader &r, const Ptr &p, int *seg, int64_t *first, int64_t *count, int *dw, int *np) {
    *count = 0;
    if (p.null) return true;
    if ((p.desc & 3) != 1 || ((p.desc >> 32) & 7) != 7) return r.fail("expected a composite list");
    const int64_t words = (int64_t)(p.desc >> 35);
    uint64_t tag;
    if (!r.word_at(p.seg, p.word, &tag)) return false;
    *count = (int64_t)((tag >> 2) & ((1ull << 30) - 1));
    *dw = (int)((tag >> 32) & 0xFFFF);
    *np = (int)(tag >> 48);
    *seg = p.seg;
    *first = p.word + 1;
    if (*count * (*dw + *np) > words || p.word + 1 + words > r.m->seg[p.seg].second) return r.fail("composite list out of bounds");
    return true;
}

template <typename F>
void parallel_for(int threads, int64_t n, F f) {
    if (threads <= 1 || n < 2) {
        f(0, n);
        return;
    }
    std::vector<std::thread> th;
    for (int t = 0; t < threads; t++) {
        const int64_t b = n * t / threads, e = n * (t + 1) / threads;
        if (b < e) th.emplace_back([=] { f(b, e); });
    }
    for (auto &x : th) x.join();
}

int parse(hymet_msh *m) {
    Reader r{m, {}};
    const uint8_t *d = m->map;
    const size_t L = m->map_len;
    HY_ARG(L >= 8, ".msh: file too short for a Cap'n Proto message");
    uint32_t nseg_m1;
    memcpy(&nseg_m1, d, 4);
    const int64_t nseg = (int64_t)nseg_m1 + 1;
    HY_ARG(nseg <= 1 << 20, ".msh: implausible segment count");
    int64_t off = 4 + 4 * nseg;
    off += (8 - off % 8) % 8;
    HY_ARG((size_t)off <= L, ".msh: truncated segment table");
    for (int64_t s = 0; s < nseg; s++) {
        uint32_t w;
        memcpy(&w, d + 4 + 4 * s, 4);
        HY_ARG((size_t)(off + 8 * (int64_t)w) <= L, ".msh: truncated segment");
        m->seg.push_back({off, (int64_t)w});
        off += 8 * (int64_t)w;
    }
    Ptr rp;
    Struct root;
    if (!r.resolve(0, 0, &rp) || !as_struct(r, rp, &root) || root.null)
        return hymet::fail(HYMET_E_ARG, ".msh: " + (r.err.empty() ? std::string("no root struct") : r.err));
    hymet_msh_info &I = m->info;
    I.k = (int32_t)data_u64(r, root, 0, 4);
    I.window_size = (int32_t)data_u64(r, root, 4, 4);
    I.sketch_size = (int32_t)data_u64(r, root, 8, 4);
    I.noncanonical = data_bit(r, root, 97);
    I.preserve_case = data_bit(r, root, 98);
    I.seed = (uint32_t)data_u64(r, root, 20, 4) ^ 42u;  // hashSeed @11 :UInt32 = 42
    I.use64 = I.k > 16;
    Ptr ap;
    if (!struct_ptr(r, root, 3, &ap) || !text(r, ap, &m->alphabet_off, &m->alphabet_len))
        return hymet::fail(HYMET_E_ARG, ".msh alphabet: " + r.err);
    // the reference list: the current one (pointer 1 or 2, whichever holds Reference
    // structs) when it has references, else referenceListOld (pointer 0)
    int rseg = 0, rdw = 0, rnp = 0;
    int64_t rfirst = 0, rcount = 0;
    for (int pi : {1, 2, 0}) {
        Ptr lp;
        Struct rl;
        if (!struct_ptr(r, root, pi, &lp) || !as_struct(r, lp, &rl)) return hymet::fail(HYMET_E_ARG, ".msh: " + r.err);
        if (rl.null) continue;
        Ptr ep;
        int sg = 0, dw = 0, np = 0;
        int64_t fst = 0, cnt = 0;
        if (!struct_ptr(r, rl, 0, &ep)) return hymet::fail(HYMET_E_ARG, ".msh: " + r.err);
        if (ep.null || (ep.desc & 3) != 1 || ((ep.desc >> 32) & 7) != 7) continue;  // not a struct list
        if (!struct_list(r, ep, &sg, &fst, &cnt, &dw, &np)) return hymet::fail(HYMET_E_ARG, ".msh: " + r.err);
        if (np == 0 || cnt == 0) continue;  // the locus list (Locus has no pointers), or empty
        rseg = sg, rfirst = fst, rcount = cnt, rdw = dw, rnp = np;
        break;
    }
    m->refs.resize((size_t)rcount);
    std::vector<std::string> errs(16);
    const int threads = (int)std::min<int64_t>(16, std::max<int64_t>(1, rcount / 4096));
    parallel_for(threads, threads, [&](int64_t tb, int64_t te) {
        for (int64_t t = tb; t < te; t++) {
            Reader rr{m, {}};
            for (int64_t i = rcount * t / threads; i < rcount * (t + 1) / threads; i++) {
                Struct s;
                s.seg = rseg;
                s.word = rfirst + i * (rdw + rnp);
                s.dwords = rdw;
                s.nptrs = rnp;
                s.null = false;
                hymet_msh::Ref &R = m->refs[(size_t)i];
                Ptr pn, pc, ph;
                const uint64_t len32 = data_u64(rr, s, 0, 4), len64 = data_u64(rr, s, 8, 8);
                R.length = (int64_t)(len64 ? len64 : len32);
                if (!struct_ptr(rr, s, 2, &pn) || !text(rr, pn, &R.name_off, &R.name_len) || !struct_ptr(rr, s, 3, &pc) ||
                    !text(rr, pc, &R.comment_off, &R.comment_len) || !struct_ptr(rr, s, I.use64 ? 5 : 4, &ph) ||
                    !prim_list(rr, ph, I.use64 ? 5 : 4, &R.hash_off, &R.n_hash)) {
                    errs[(size_t)t] = rr.err;
                    return;
                }
            }
        }
    });
    for (auto &e : errs)
        if (!e.empty()) return hymet::fail(HYMET_E_ARG, ".msh reference: " + e);
    I.n_refs = rcount;
    int64_t nh = 0, nb = 0, cb = 0;
    for (auto &R : m->refs) {
        nh += R.n_hash;
        nb += R.name_len + 1;
        cb += R.comment_len + 1;
    }
    I.n_hashes = nh;
    I.names_bytes = nb;
    I.comments_bytes = cb;
    I.alphabet_len = m->alphabet_len;
    return HYMET_OK;
}

// dst_all[lo_h, hi_h) = hashes [lo_h, hi_h) of the concatenation (off: n_refs + 1 hash
// offsets), `threads` host threads over equal hash counts; 32-bit sketches widened, any list
// that is not ascending sorted; a reference straddling a thread's or the range's bounds is
// gathered (and sorted if need be) whole into a scratch list and copied in part
void gather_hashes(const hymet_msh *m, const std::vector<int64_t> &off, int64_t lo_h, int64_t hi_h, int threads,
                   uint64_t *dst_all) {
    const int64_t n = m->info.n_refs, span = hi_h - lo_h;
    if (span <= 0 || n <= 0) return;
    if (span < (1 << 20)) threads = 1;
    const bool use64 = m->info.use64;
    parallel_for(threads, threads, [&](int64_t tb, int64_t te) {
        std::vector<uint64_t> tmp;
        for (int64_t t = tb; t < te; t++) {
            const int64_t a = lo_h + span * t / threads, b = lo_h + span * (t + 1) / threads;
            if (a >= b) continue;
            // the reference holding hash a: the last one starting at or before it
            int64_t i = std::upper_bound(off.begin(), off.begin() + n + 1, a) - off.begin() - 1;
            for (; i < n && off[(size_t)i] < b; i++) {
                const auto &R = m->refs[(size_t)i];
                const int64_t r0 = off[(size_t)i], r1 = off[(size_t)i + 1];
                const int64_t s = std::max(a, r0), e = std::min(b, r1);
                if (s >= e) continue;
                const bool whole = s == r0 && e == r1;
                if (!whole) tmp.resize((size_t)R.n_hash);
                uint64_t *dst = whole ? dst_all + r0 : tmp.data();
                if (use64) {
                    memcpy(dst, m->map + R.hash_off, 8 * (size_t)R.n_hash);
                } else {
                    const uint8_t *src = m->map + R.hash_off;
                    for (int64_t j = 0; j < R.n_hash; j++) {
                        uint32_t v;
                        memcpy(&v, src + 4 * j, 4);
                        dst[j] = v;
                    }
                }
                if (!std::is_sorted(dst, dst + R.n_hash)) std::sort(dst, dst + R.n_hash);
                if (!whole) memcpy(dst_all + s, dst + (s - r0), 8 * (size_t)(e - s));
            }
        }
    });
}

// start of each reference's name / comment in the NUL-separated pools (n + 1 entries each)
void text_offsets(const hymet_msh *m, int64_t *name_start, int64_t *comment_start) {
    const int64_t n = m->info.n_refs;
    name_start[0] = comment_start[0] = 0;
    for (int64_t i = 0; i < n; i++) {
        name_start[i + 1] = name_start[i] + m->refs[(size_t)i].name_len + 1;
        comment_start[i + 1] = comment_start[i] + m->refs[(size_t)i].comment_len + 1;
    }
}

}  // namespace

extern "C" {

int hymet_msh_text_offsets(const hymet_msh *m, int64_t *name_start, int64_t *comment_start) {
    HY_ARG(m && name_start && comment_start, "hymet_msh_text_offsets: null argument");
    text_offsets(m, name_start, comment_start);
    return HYMET_OK;
}

int hymet_msh_open(const char *path, hymet_msh **out) {
    HY_ARG(path && out, "hymet_msh_open: null argument");
    *out = nullptr;
    const int fd = open(path, O_RDONLY);
    if (fd < 0) return hymet::fail(HYMET_E_ARG, std::string("hymet_msh_open: cannot open ") + path);
    struct stat st;
    if (fstat(fd, &st) != 0 || st.st_size <= 0) {
        close(fd);
        return hymet::fail(HYMET_E_ARG, std::string("hymet_msh_open: empty or unreadable ") + path);
    }
    void *p = mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_PRIVATE, fd, 0);
    close(fd);
    if (p == MAP_FAILED) return hymet::fail(HYMET_E_ARG, std::string("hymet_msh_open: mmap failed for ") + path);
    auto *m = new hymet_msh;
    m->map = (const uint8_t *)p;
    m->map_len = (size_t)st.st_size;
    const int rc = parse(m);
    if (rc) {
        hymet_msh_close(m);
        return rc;
    }
    *out = m;
    return HYMET_OK;
}

int hymet_msh_info_get(const hymet_msh *m, hymet_msh_info *info) {
    HY_ARG(m && info, "hymet_msh_info_get: null argument");
    *info = m->info;
    return HYMET_OK;
}

int hymet_msh_copy(const hymet_msh *m, int threads, uint64_t *hashes, int64_t *offsets, int64_t *lengths, char *names,
                   char *comments, char *alphabet) {
    HY_ARG(m, "hymet_msh_copy: null handle");
    const int64_t n = m->info.n_refs;
    if (offsets) {
        offsets[0] = 0;
        for (int64_t i = 0; i < n; i++) offsets[i + 1] = offsets[i] + m->refs[(size_t)i].n_hash;
    }
    if (lengths)
        for (int64_t i = 0; i < n; i++) lengths[i] = m->refs[(size_t)i].length;
    // names / comments: NUL-separated, in reference order; the texts lie scattered through the
    // mapped file (a page fault and a cache miss or two each), so threads take reference ranges
    if (names || comments) {
        std::vector<int64_t> no((size_t)n + 1, 0), co((size_t)n + 1, 0);
        text_offsets(m, no.data(), co.data());
        const int th = (int)std::max<int64_t>(1, std::min<int64_t>({(int64_t)std::max(threads, 1), 16, n / 2048}));
        parallel_for(th, n, [&](int64_t b, int64_t e) {
            for (int64_t i = b; i < e; i++) {
                const auto &R = m->refs[(size_t)i];
                if (names) {
                    if (R.name_len) memcpy(names + no[(size_t)i], m->map + R.name_off, (size_t)R.name_len);
                    names[no[(size_t)i] + R.name_len] = 0;
                }
                if (comments) {
                    if (R.comment_len) memcpy(comments + co[(size_t)i], m->map + R.comment_off, (size_t)R.comment_len);
                    comments[co[(size_t)i] + R.comment_len] = 0;
                }
            }
        });
    }
    if (alphabet && m->alphabet_len) memcpy(alphabet, m->map + m->alphabet_off, (size_t)m->alphabet_len);
    if (!hashes || n == 0) return HYMET_OK;
    // hashes: threads take contiguous reference ranges of about equal hash counts
    std::vector<int64_t> off((size_t)n + 1, 0);
    for (int64_t i = 0; i < n; i++) off[(size_t)i + 1] = off[(size_t)i] + m->refs[(size_t)i].n_hash;
    threads = std::max(1, std::min(threads, 64));
    const int64_t total = off[(size_t)n];
    if (total < (1 << 20)) threads = 1;
    gather_hashes(m, off, 0, total, threads, hashes);
    return HYMET_OK;
}

int hymet_msh_upload_range(hymet_ctx *ctx, const hymet_msh *m, int threads, uint64_t *pinned, uint64_t *d_hashes,
                           int n_chunks, int64_t lo_h, int64_t hi_h) {
    HY_ARG(ctx && m, "hymet_msh_upload_range: null argument");
    const int64_t n = m->info.n_refs;
    HY_ARG(lo_h >= 0 && lo_h <= hi_h && hi_h <= m->info.n_hashes, "hymet_msh_upload_range: bad hash range");
    if (n == 0 || lo_h == hi_h) return HYMET_OK;
    HY_ARG(pinned && d_hashes, "hymet_msh_upload_range: null buffer");
    HY_HIP(hipSetDevice(ctx->device));
    std::vector<int64_t> off((size_t)n + 1, 0);
    for (int64_t i = 0; i < n; i++) off[(size_t)i + 1] = off[(size_t)i] + m->refs[(size_t)i].n_hash;
    threads = std::max(1, std::min(threads, 64));
    n_chunks = std::max(1, std::min(n_chunks, 64));
    const int64_t span = hi_h - lo_h;
    if (span < (1 << 20)) threads = 1;
    // equal hash counts per chunk.  One set of threads walks the chunks in order, each taking
    // its share of every chunk; the caller queues a chunk's DMA as soon as every thread is
    // past it (threads spawned once: per-chunk spawns cost more than a small slice's copy)
    std::unique_ptr<std::atomic<int>[]> done(new std::atomic<int>[(size_t)n_chunks]);
    for (int c = 0; c < n_chunks; c++) done[(size_t)c].store(0);
    auto chunk = [&](int c, int64_t *lo, int64_t *hi) {
        *lo = lo_h + span * c / n_chunks;
        *hi = lo_h + span * (c + 1) / n_chunks;
    };
    std::vector<std::thread> th;
    for (int t = 0; t < threads; t++)
        th.emplace_back([&, t] {
            for (int c = 0; c < n_chunks; c++) {
                int64_t lo, hi;
                chunk(c, &lo, &hi);
                gather_hashes(m, off, lo + (hi - lo) * t / threads, lo + (hi - lo) * (t + 1) / threads, 1, pinned);
                done[(size_t)c].fetch_add(1, std::memory_order_release);
            }
        });
    hipError_t err = hipSuccess;
    for (int c = 0; c < n_chunks; c++) {
        while (done[(size_t)c].load(std::memory_order_acquire) < threads) std::this_thread::yield();
        int64_t lo, hi;
        chunk(c, &lo, &hi);
        if (hi > lo && err == hipSuccess)
            err = hipMemcpyAsync(d_hashes + lo, pinned + lo, 8 * (size_t)(hi - lo), hipMemcpyHostToDevice, ctx->stream);
    }
    for (auto &x : th) x.join();
    HY_HIP(err);
    return HYMET_OK;
}

int hymet_msh_upload(hymet_ctx *ctx, const hymet_msh *m, int threads, uint64_t *pinned, uint64_t *d_hashes,
                     int n_chunks) {
    HY_ARG(ctx && m && (m->info.n_hashes == 0 || (pinned && d_hashes)), "hymet_msh_upload: null argument");
    return hymet_msh_upload_range(ctx, m, threads, pinned, d_hashes, n_chunks, 0, m->info.n_hashes);
}

void hymet_msh_close(hymet_msh *m) {
    if (!m) return;
    if (m->map) munmap((void *)m->map, m->map_len);
    delete m;
}

}  // extern "C"
