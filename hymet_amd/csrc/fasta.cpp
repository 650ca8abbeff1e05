// Host half of the FASTA ingest: the record table of a FASTA file held in host memory.
//
// The reference hands the pooled contigs to Mash and minimap2 as files (scripts/mash.sh:14,
// scripts/minimap2.sh:23), whose kseq readers cut records at '>' starting a line; the name is
// the header's first whitespace-delimited token and the sequence is the following lines with
// line breaks removed.  This scan finds, for every record, the byte ranges the device needs
// (name, sequence) and the base count, on `threads` host threads.  No sequence byte is
// copied: the device half (ingest.hip) uploads one contiguous byte range of the file and
// strips the line breaks there.  Semantics equal hymet_amd.seqio.parse_fasta_bytes.
#include "common.hpp"

#include <algorithm>
#include <cstring>
#include <thread>
#include <vector>

namespace {

inline bool is_ws(unsigned char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' || c == '\f'; }

// record starts ('>' at the start of the buffer or right after '\n') in [b, e)
void find_starts(const char *buf, int64_t b, int64_t e, std::vector<int64_t> &out) {
    int64_t p = b;
    while (p < e) {
        const void *q = memchr(buf + p, '>', (size_t)(e - p));
        if (!q) break;
        const int64_t i = (const char *)q - buf;
        if (i == 0 || buf[i - 1] == '\n') out.push_back(i);
        p = i + 1;
    }
}

// exact count of zero bytes in a 64-bit word (no borrow false positives)
inline int zero_bytes(uint64_t v) {
    const uint64_t m = 0x7F7F7F7F7F7F7F7Full;
    return __builtin_popcountll(~(((v & m) + m) | v | m));
}

// '\n' and '\r' bytes in s[0, n): 8 bytes per step (SWAR), ~8x the byte loop
int64_t count_breaks(const char *s, int64_t n) {
    int64_t c = 0, i = 0;
    for (; i < n && ((uintptr_t)(s + i) & 7); i++) c += (s[i] == '\n') | (s[i] == '\r');
    const uint64_t nl = 0x0A0A0A0A0A0A0A0Aull, cr = 0x0D0D0D0D0D0D0D0Dull;
    for (; i + 8 <= n; i += 8) {
        uint64_t w;
        memcpy(&w, s + i, 8);
        c += zero_bytes(w ^ nl) + zero_bytes(w ^ cr);
    }
    for (; i < n; i++) c += (s[i] == '\n') | (s[i] == '\r');
    return c;
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

}  // namespace

extern "C" int hymet_fasta_index(const char *h_buf, int64_t n, int threads, int64_t cap, int64_t *n_rec,
                                 int64_t *h_name_off, int32_t *h_name_len, int64_t *h_seq_off, int64_t *h_seq_end,
                                 int64_t *h_nbases) {
    HY_ARG(n_rec && (n == 0 || h_buf), "hymet_fasta_index: null argument");
    HY_ARG(n >= 0 && cap >= 0, "hymet_fasta_index: negative size");
    threads = std::max(1, std::min(threads, 64));
    if (n < (int64_t)1 << 22) threads = 1;
    // 1 record starts, in parallel over byte ranges
    std::vector<std::vector<int64_t>> part(threads);
    parallel_for(threads, threads, [&](int64_t b, int64_t e) {
        for (int64_t t = b; t < e; t++) find_starts(h_buf, n * t / threads, n * (t + 1) / threads, part[t]);
    });
    std::vector<int64_t> st;
    for (auto &v : part) st.insert(st.end(), v.begin(), v.end());
    const int64_t R = (int64_t)st.size();
    *n_rec = R;
    if (R > cap) return hymet::fail(HYMET_E_CAPACITY, "hymet_fasta_index: more records than cap");
    HY_ARG(R == 0 || (h_name_off && h_name_len && h_seq_off && h_seq_end && h_nbases), "hymet_fasta_index: null output");
    // 2 per record: header line, name token, sequence range and base count, in parallel
    // over records (a record's sequence is scanned once for line breaks)
    parallel_for(threads, R, [&](int64_t b, int64_t e) {
        for (int64_t r = b; r < e; r++) {
            const int64_t s = st[r] + 1;                            // after '>'
            const int64_t end = r + 1 < R ? st[r + 1] - 1 : n;      // the '\n' before the next '>'
            const void *nl = memchr(h_buf + s, '\n', (size_t)std::max<int64_t>(0, end - s));
            const int64_t hend = nl ? (const char *)nl - h_buf : end;
            int64_t a = s;
            while (a < hend && is_ws((unsigned char)h_buf[a])) a++;
            int64_t z = a;
            while (z < hend && !is_ws((unsigned char)h_buf[z])) z++;
            h_name_off[r] = a;
            h_name_len[r] = (int32_t)(z - a);
            const int64_t so = nl ? hend + 1 : end;
            h_seq_off[r] = so;
            h_seq_end[r] = end;
            h_nbases[r] = (end - so) - count_breaks(h_buf + so, end - so);
        }
    });
    return HYMET_OK;
}

// names of n records gathered into one pool (h_pool_off: n + 1 offsets, computed here)
extern "C" int hymet_fasta_names(const char *h_buf, const int64_t *h_name_off, const int32_t *h_name_len, int64_t n,
                                 char *h_pool, int64_t *h_pool_off) {
    HY_ARG(n == 0 || (h_buf && h_name_off && h_name_len && h_pool && h_pool_off), "hymet_fasta_names: null argument");
    if (n <= 0) {
        if (h_pool_off) h_pool_off[0] = 0;
        return HYMET_OK;
    }
    h_pool_off[0] = 0;
    for (int64_t i = 0; i < n; i++) h_pool_off[i + 1] = h_pool_off[i] + h_name_len[i];
    for (int64_t i = 0; i < n; i++) memcpy(h_pool + h_pool_off[i], h_buf + h_name_off[i], (size_t)h_name_len[i]);
    return HYMET_OK;
}
