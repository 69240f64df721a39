// layout_bench.hip — pure data-movement model of one fused tile pass at n qubits (no gates, no
// LDS): each 256-thread workgroup moves one 12-qubit tile of 4096 amplitudes, lanes = tile bits
// 0..5, waves = tile bits 6..7, 16 registers = tile bits 8..11 (the pass kernels' first / last
// stage pattern).  Reads with tile layout R from `src`, writes with tile layout W to `dst`
// (in place when R == W and src == dst).  Tile ids enumerate the non-tile qubits in ascending
// order; workgroups map to tile ids XCD-contiguously (QSIM_JIT_XCD = 1) or naturally.
//
// build: hipcc -O3 --offload-arch=gfx950 -o layout_bench layout_bench.hip
// usage: ./layout_bench n < configs      config line: "r0,r1,...,r11 w0,...,w11 order inplace"
// prints one JSON line per config: ms per pass, GB/s (32 B per amplitude).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <sstream>
#include <string>
#include <vector>

#define CHK(x)                                                                  \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            std::fprintf(stderr, "%s at %d\n", hipGetErrorString(e), __LINE__); \
            std::exit(1);                                                       \
        }                                                                       \
    } while (0)

struct Layout {
    unsigned long long tbit[12];  // address bit (amplitude index) of each tile bit
    unsigned long long zmask;     // tile positions (skipped by the tile-id deposit)
};
struct Args {
    Layout r, w;
    int order;  // 0 natural, 1 XCD-contiguous
    int rot;    // tile id = rotate-left of the (ordered) block index by rot within log2(grid) bits
    int tbits;
    int policy;  // bit 0: temporal loads, bit 1: temporal stores (default non-temporal)
    unsigned long long swz[64];  // physical address = index ^ XOR of swz[q] over its set bits q
};

__device__ __forceinline__ unsigned long long deposit(unsigned long long k, unsigned long long zmask) {
    for (unsigned long long m = zmask; m; m &= m - 1ull) {
        const unsigned long long lo = k & ((1ull << __builtin_ctzll(m)) - 1ull);
        k = ((k ^ lo) << 1) | lo;
    }
    return k;
}

typedef double qdv2 __attribute__((ext_vector_type(2)));

__global__ void __launch_bounds__(256, 2) k_move(const double2* __restrict__ src, double2* __restrict__ dst,
                                                 Args a) {
    const unsigned long long b = blockIdx.x;
    unsigned long long tile =
        (a.order == 1 && (gridDim.x & 7u) == 0) ? (b & 7ull) * (gridDim.x >> 3) + (b >> 3) : b;
    if (a.rot) tile = ((tile << a.rot) | (tile >> (a.tbits - a.rot))) & ((1ull << a.tbits) - 1ull);
    unsigned long long rbase = deposit(tile, a.r.zmask), wbase = deposit(tile, a.w.zmask);
    {
        unsigned long long x = 0, y = 0;
        for (unsigned long long m = rbase; m; m &= m - 1ull) x ^= a.swz[__builtin_ctzll(m)];
        for (unsigned long long m = wbase; m; m &= m - 1ull) y ^= a.swz[__builtin_ctzll(m)];
        rbase ^= x;
        wbase ^= y;
    }
    const unsigned t = threadIdx.x;
    unsigned long long ro = rbase, wo = wbase;
#pragma unroll
    for (int i = 0; i < 8; ++i)
        if ((t >> i) & 1u) {
            ro ^= a.r.tbit[i];
            wo ^= a.w.tbit[i];
        }
    qdv2 v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        unsigned long long o = ro;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if ((r >> i) & 1) o ^= a.r.tbit[8 + i];
        if (a.policy & 1) v[r] = *reinterpret_cast<const qdv2*>(src + o);
        else v[r] = __builtin_nontemporal_load(reinterpret_cast<const qdv2*>(src + o));
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        unsigned long long o = wo;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if ((r >> i) & 1) o ^= a.w.tbit[8 + i];
        if (a.policy & 2) *reinterpret_cast<qdv2*>(dst + o) = v[r];
        else __builtin_nontemporal_store(v[r], reinterpret_cast<qdv2*>(dst + o));
    }
}

static unsigned long long g_swz[64];
static Layout make_layout(const std::vector<int>& pos) {
    Layout l{};
    for (int i = 0; i < 12; ++i) {
        l.tbit[i] = (1ull << pos[i]) ^ g_swz[pos[i]];
        l.zmask |= 1ull << pos[i];
    }
    return l;
}
static std::vector<int> parse_list(const std::string& s) {
    std::vector<int> v;
    std::stringstream ss(s);
    std::string x;
    while (std::getline(ss, x, ',')) v.push_back(std::atoi(x.c_str()));
    return v;
}

int main(int argc, char** argv) {
    const int n = argc > 1 ? std::atoi(argv[1]) : 30;
    const int reps = argc > 2 ? std::atoi(argv[2]) : 5;
    const size_t N = 1ull << n;
    double2 *a = nullptr, *b = nullptr;
    CHK(hipMalloc(&a, N * sizeof(double2)));
    CHK(hipMalloc(&b, N * sizeof(double2)));
    CHK(hipMemset(a, 0, N * sizeof(double2)));
    CHK(hipMemset(b, 0, N * sizeof(double2)));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    const unsigned grid = (unsigned)(N >> 12);
    int order = 1, inplace = 1;
    char line[512];
    while (std::fgets(line, sizeof line, stdin)) {
        char r[200], w[200];
        int rot = 0, policy = 0;
        unsigned swzseed = 0;
        int swzlo = 6, swzw = 6;
        if (std::sscanf(line, "%199s %199s %d %d %d %d %u %d %d", r, w, &order, &inplace, &rot, &policy, &swzseed,
                        &swzlo, &swzw) < 4)
            continue;
        // swizzle: every index bit q >= swzlo + swzw also flips a pseudo-random pattern of bits
        // [swzlo, swzlo + swzw) (unitriangular, so a bijection)
        for (int q = 0; q < 64; ++q) {
            g_swz[q] = 0;
            if (swzseed && q >= swzlo + swzw && q < n) {
                unsigned long long h = (unsigned long long)swzseed * 0x9E3779B97F4A7C15ull + (unsigned long long)q * 0xBF58476D1CE4E5B9ull;
                h ^= h >> 31;
                h *= 0x94D049BB133111EBull;
                h ^= h >> 29;
                g_swz[q] = (h & ((1ull << swzw) - 1ull)) << swzlo;
            }
        }
        const std::vector<int> rp = parse_list(r), wp = parse_list(w);
        if (rp.size() != 12 || wp.size() != 12) continue;
        unsigned long long mr = 0, mw = 0;  // distinct positions below n, or the line is skipped
        for (int i = 0; i < 12; ++i) {
            if (rp[i] < 0 || rp[i] >= n || wp[i] < 0 || wp[i] >= n) mr = mw = ~0ull;
            else {
                mr |= 1ull << rp[i];
                mw |= 1ull << wp[i];
            }
        }
        if (__builtin_popcountll(mr) != 12 || __builtin_popcountll(mw) != 12) continue;
        Args args{make_layout(rp), make_layout(wp), order, rot, n - 12, policy, {}};
        for (int q = 0; q < 64; ++q) args.swz[q] = g_swz[q];
        double2* src = a;
        double2* dst = inplace ? a : b;
        k_move<<<grid, 256>>>(src, dst, args);  // warm
        CHK(hipDeviceSynchronize());
        CHK(hipEventRecord(e0));
        for (int i = 0; i < reps; ++i) k_move<<<grid, 256>>>(src, dst, args);
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        float ms = 0;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        std::printf("{\"r\": [%s], \"w\": [%s], \"order\": %d, \"inplace\": %d, \"rot\": %d, \"policy\": %d, \"swz\": [%u, %d, %d], \"ms\": %.4f, \"GBps\": %.1f}\n", r,
                    w, order, inplace, rot, policy, swzseed, swzlo, swzw, ms, 32.0 * N / (ms * 1e-3) / 1e9);
        std::fflush(stdout);
    }
    return 0;
}
