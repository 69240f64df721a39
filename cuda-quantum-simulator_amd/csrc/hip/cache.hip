// cache.hip — an on-disk cache across processes for the two first-run costs of a circuit:
// the circuit-specialised pass kernels (hipRTC code objects, jit.hip) and the layout decisions
// (relabeling / relayout / tile height, possibly timed on the device: relabel.hip's memo).
//
// A new process running a circuit it (or another process on this machine) ran before loads the
// code objects instead of compiling them (≈0.5-1 s each) and takes the memoised layout instead of
// planning and timing the candidates again ("calibration results are not reused across
// processes").  Entries are verified in full before use (the memo stores its whole key; code
// objects are keyed by two independent 64-bit hashes of the generated source, the compile
// options and this library's build stamp), written atomically (temporary file + rename), and any
// I/O failure is a cache miss.  QSIM_CACHE=0 turns it off; QSIM_CACHE_DIR sets the directory
// (default $XDG_CACHE_HOME/qsim_amd, else $HOME/.cache/qsim_amd).
#include <sys/stat.h>
#include <sys/types.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <thread>
#include <vector>

#include "engine.hpp"
#include "qsim_hip.h"

namespace qsim_hip {

static std::atomic<uint64_t> g_jit_hits{0}, g_jit_stores{0}, g_memo_hits{0}, g_memo_stores{0};

// this library's build stamp: entries of another build are misses (the planner may differ)
static const char* build_stamp() { return __DATE__ " " __TIME__; }

static bool mkdirs(const std::string& d) {
    if (d.empty()) return false;
    std::string cur;
    for (size_t i = 0; i <= d.size(); ++i) {
        if (i == d.size() || d[i] == '/') {
            if (!cur.empty() && ::mkdir(cur.c_str(), 0755) != 0 && errno != EEXIST) return false;
        }
        if (i < d.size()) cur.push_back(d[i]);
    }
    struct stat st;
    return ::stat(d.c_str(), &st) == 0 && S_ISDIR(st.st_mode);
}

// The cache directory, or "" when the cache is off or unusable (read per call: tests switch it).
std::string cache_dir() {
    const char* on = std::getenv("QSIM_CACHE");
    if (on && std::atoi(on) == 0) return "";
    std::string d;
    if (const char* e = std::getenv("QSIM_CACHE_DIR")) {
        d = e;
    } else if (const char* x = std::getenv("XDG_CACHE_HOME")) {
        d = std::string(x) + "/qsim_amd";
    } else if (const char* h = std::getenv("HOME")) {
        d = std::string(h) + "/.cache/qsim_amd";
    }
    return mkdirs(d) ? d : "";
}

uint64_t cache_hash(const void* p, size_t n, uint64_t seed) {  // FNV-1a with a seed, then a mixer
    const unsigned char* b = static_cast<const unsigned char*>(p);
    uint64_t h = 0xcbf29ce484222325ull ^ (seed * 0x9e3779b97f4a7c15ull);
    for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 0x100000001b3ull;
    h ^= h >> 33;
    h *= 0xff51afd7ed558ccdull;
    h ^= h >> 33;
    return h;
}

static bool read_file(const std::string& path, std::vector<char>& out) {
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) return false;
    std::vector<char> buf;
    char tmp[1 << 16];
    size_t r;
    while ((r = std::fread(tmp, 1, sizeof tmp, f)) > 0) buf.insert(buf.end(), tmp, tmp + r);
    const bool ok = !std::ferror(f);
    std::fclose(f);
    if (ok) out.swap(buf);
    return ok;
}

static bool write_file_atomic(const std::string& path, const std::vector<char>& data) {
    const std::string tmp = path + ".tmp." + std::to_string((long)::getpid()) + "." +
                            std::to_string(std::hash<std::thread::id>{}(std::this_thread::get_id()));
    FILE* f = std::fopen(tmp.c_str(), "wb");
    if (!f) return false;
    const bool ok = std::fwrite(data.data(), 1, data.size(), f) == data.size();
    if (std::fclose(f) != 0 || !ok || std::rename(tmp.c_str(), path.c_str()) != 0) {
        (void)std::remove(tmp.c_str());
        return false;
    }
    return true;
}

static std::string hex(uint64_t v) {
    char b[17];
    std::snprintf(b, sizeof b, "%016llx", (unsigned long long)v);
    return b;
}

// ---- code objects ----
// header: magic, stamp hash, source length, both source hashes; then the code object
namespace {
struct JitHdr {
    char magic[8];
    uint64_t stamp, len, h1, h2, code_len;
};
}  // namespace

static uint64_t opts_stamp(const std::string& opts) {
    const std::string s = std::string(build_stamp()) + "|" + opts;
    return cache_hash(s.data(), s.size(), 7);
}

bool jit_cache_load(const std::string& src, const std::string& opts, std::vector<char>& code) {
    const std::string d = cache_dir();
    if (d.empty()) return false;
    const uint64_t h1 = cache_hash(src.data(), src.size(), 1), h2 = cache_hash(src.data(), src.size(), 2);
    std::vector<char> buf;
    if (!read_file(d + "/jit_" + hex(h1 ^ opts_stamp(opts)) + ".co", buf) || buf.size() < sizeof(JitHdr)) return false;
    JitHdr hd;
    std::memcpy(&hd, buf.data(), sizeof hd);
    if (std::memcmp(hd.magic, "QSIMJIT1", 8) != 0 || hd.stamp != opts_stamp(opts) || hd.len != src.size() ||
        hd.h1 != h1 || hd.h2 != h2 || hd.code_len == 0 || buf.size() != sizeof hd + hd.code_len)
        return false;
    code.assign(buf.begin() + sizeof hd, buf.end());
    ++g_jit_hits;
    return true;
}

void jit_cache_store(const std::string& src, const std::string& opts, const std::vector<char>& code) {
    const std::string d = cache_dir();
    if (d.empty() || code.empty()) return;
    JitHdr hd;
    std::memcpy(hd.magic, "QSIMJIT1", 8);
    hd.stamp = opts_stamp(opts);
    hd.len = src.size();
    hd.h1 = cache_hash(src.data(), src.size(), 1);
    hd.h2 = cache_hash(src.data(), src.size(), 2);
    hd.code_len = code.size();
    std::vector<char> buf(sizeof hd);
    std::memcpy(buf.data(), &hd, sizeof hd);
    buf.insert(buf.end(), code.begin(), code.end());
    if (write_file_atomic(d + "/jit_" + hex(hd.h1 ^ hd.stamp) + ".co", buf)) ++g_jit_stores;
}

// ---- layout decisions ----
// n, kind (relabel.hip's extended kind), the full key, h, perm, the build stamp
static std::vector<char> memo_record(int n, int kind, const void* key, size_t bytes, int h,
                                     const std::vector<int>& perm) {
    std::vector<char> b;
    auto put = [&](const void* p, size_t k) {
        const char* c = static_cast<const char*>(p);
        b.insert(b.end(), c, c + k);
    };
    const char magic[8] = {'Q', 'S', 'I', 'M', 'M', 'E', 'M', '1'};
    put(magic, 8);
    const std::string st = build_stamp();
    const uint32_t sl = (uint32_t)st.size(), pl = (uint32_t)perm.size();
    const uint64_t kb = bytes;
    put(&sl, 4);
    put(st.data(), sl);
    put(&n, 4);
    put(&kind, 4);
    put(&h, 4);
    put(&pl, 4);
    if (pl) put(perm.data(), pl * sizeof(int));
    put(&kb, 8);
    put(key, bytes);
    return b;
}
static std::string memo_path(const std::string& d, int n, int kind, const void* key, size_t bytes) {
    return d + "/memo_" + hex(cache_hash(key, bytes, 3) ^ ((uint64_t)n << 40) ^ ((uint64_t)(uint32_t)kind << 8)) +
           ".lay";
}

bool layout_cache_load(int n, int kind, const void* key, size_t bytes, std::vector<int>& perm, int* h) {
    const std::string d = cache_dir();
    if (d.empty()) return false;
    std::vector<char> buf;
    if (!read_file(memo_path(d, n, kind, key, bytes), buf)) return false;
    // parse: the record must equal one made from the same key, up to h and perm
    size_t o = 0;
    auto get = [&](void* p, size_t k) {
        if (o + k > buf.size()) return false;
        std::memcpy(p, buf.data() + o, k);
        o += k;
        return true;
    };
    char magic[8];
    uint32_t sl = 0, pl = 0;
    int rn = 0, rk = 0, rh = -1;
    uint64_t kb = 0;
    if (!get(magic, 8) || std::memcmp(magic, "QSIMMEM1", 8) != 0 || !get(&sl, 4) || sl > 256) return false;
    std::string st(sl, '\0');
    if (!get(&st[0], sl) || st != build_stamp() || !get(&rn, 4) || !get(&rk, 4) || !get(&rh, 4) || !get(&pl, 4) ||
        rn != n || rk != kind || pl > 64)
        return false;
    std::vector<int> p(pl);
    if ((pl && !get(p.data(), pl * sizeof(int))) || !get(&kb, 8) || kb != bytes || o + bytes != buf.size() ||
        std::memcmp(buf.data() + o, key, bytes) != 0)
        return false;
    for (int x : p)
        if (x < 0 || x >= n) return false;
    perm = std::move(p);
    if (h) *h = rh;
    ++g_memo_hits;
    return true;
}

void layout_cache_store(int n, int kind, const void* key, size_t bytes, int h, const std::vector<int>& perm) {
    const std::string d = cache_dir();
    if (d.empty()) return;
    if (write_file_atomic(memo_path(d, n, kind, key, bytes), memo_record(n, kind, key, bytes, h, perm)))
        ++g_memo_stores;
}

}  // namespace qsim_hip

extern "C" int qsim_cache_stats(uint64_t* jit_hits, uint64_t* jit_stores, uint64_t* layout_hits,
                                uint64_t* layout_stores) {
    using namespace qsim_hip;
    if (jit_hits) *jit_hits = g_jit_hits.load();
    if (jit_stores) *jit_stores = g_jit_stores.load();
    if (layout_hits) *layout_hits = g_memo_hits.load();
    if (layout_stores) *layout_stores = g_memo_stores.load();
    return QSIM_OK;
}
