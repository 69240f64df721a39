// jit.hip — circuit-specialised fused-pass kernels (hipRTC), the second execution tier.
//
// The staged pass interpreter (fused.hip, k_fused_staged) dispatches every op at run time: a
// scalar descriptor load, a branch tree on (kind, sub, register bit) and, because the branch arms
// produce their register arrays in different VGPRs, v_mov copies of the live amplitudes at every
// merge.  For deep passes that VALU overhead, not HBM, bounds the pass.
//
// Here the same Plan is printed as straight-line HIP: one kernel per staged pass, every op
// expanded over its 2^rb register pairs with the target bit, register-bit controls and matrix
// entries as literals (hex-float, exact), uncontrolled X gates as pure register renames, and the
// load / LDS / store addressing of each stage as constants.  The source is compiled by hipRTC for
// gfx950 on a background thread the first time a plan is seen; until the code object is ready
// the interpreter runs the plan (so a one-shot circuit never waits for the compiler), and from
// then on the state's runs of that plan launch the specialised kernels.  Semantics are those of
// the interpreter op for op (same unnormalised-H scale, same closed forms as device_ops.hpp).
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <memory>
#include <mutex>
#include <sstream>
#include <thread>

#include "engine.hpp"

namespace qsim_hip {

// ---------------------------------------------------------------------------------------
// Policy
// ---------------------------------------------------------------------------------------
static std::atomic<int> g_jit_mode{-1};        // 0 off, 1 background compile, 2 compile inline
static std::atomic<int> g_jit_min_qubits{-1};  // smaller states always use the interpreter

static int env_or(const char* k, int d) {
    const char* e = std::getenv(k);
    return e ? std::atoi(e) : d;
}
int jit_mode() {
    int m = g_jit_mode.load();
    if (m < 0) {
        m = env_or("QSIM_JIT", 1);
        g_jit_mode.store(m);
    }
    return m;
}
int jit_min_qubits() {
    int m = g_jit_min_qubits.load();
    if (m < 0) {
        m = env_or("QSIM_JIT_MIN_QUBITS", 20);
        g_jit_min_qubits.store(m);
    }
    return m;
}
void jit_configure(int mode, int min_qubits) {
    if (mode >= 0) g_jit_mode.store(mode);
    if (min_qubits >= 0) g_jit_min_qubits.store(min_qubits);
}

// ---------------------------------------------------------------------------------------
// Source generation
// ---------------------------------------------------------------------------------------
namespace {

std::string lit(double x) {  // exact double literal
    char b[64];
    std::snprintf(b, sizeof b, "%a", x);
    return b;
}
std::string hexu(uint64_t x) {
    char b[32];
    std::snprintf(b, sizeof b, "0x%llxull", (unsigned long long)x);
    return b;
}

// HBM access of the generated passes: non-temporal by default (a pass touches every amplitude
// once); QSIM_JIT_NT=0 uses the default cache policy (Infinity Cache residency experiments).
const char* kPreludeNT = R"(
typedef double qdv2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ double2 qld(const double2* p) {
  const qdv2 t = __builtin_nontemporal_load(reinterpret_cast<const qdv2*>(p));
  return make_double2(t.x, t.y);
}
__device__ __forceinline__ void qst(double2* p, double2 v) {
  qdv2 t; t.x = v.x; t.y = v.y;
  __builtin_nontemporal_store(t, reinterpret_cast<qdv2*>(p));
}
)";
const char* kPreludeT = R"(
__device__ __forceinline__ double2 qld(const double2* p) { return *p; }
__device__ __forceinline__ void qst(double2* p, double2 v) { *p = v; }
)";
const char* kPrelude = R"(
__device__ __forceinline__ double2 qsel(bool c, double2 a, double2 b) {
  return make_double2(c ? a.x : b.x, c ? a.y : b.y);
}
__device__ __forceinline__ double2 qcm(double mr, double mi, double2 a) {
  return make_double2(mr * a.x - mi * a.y, mr * a.y + mi * a.x);
}
__device__ __forceinline__ unsigned qins0(unsigned p, int b) {
  const unsigned lo = p & ((1u << b) - 1u);
  return ((p ^ lo) << 1) | lo;
}
)";

struct Gen {
    std::ostringstream o;
    int R = 16, RB = 4;
    int nm[16];  // logical register r lives in variable v<nm[r]>
    int tmp = 0;

    std::string v(int r) const { return "v" + std::to_string(nm[r]); }

    // |1>-side phase of a diagonal op (diag1 in device_ops.hpp)
    std::string diag1(const TileOp& t, const std::string& a) {
        const double c = kInvSqrt2;
        switch (t.sub) {
            case S_NEG: return "make_double2(-" + a + ".x, -" + a + ".y)";
            case S_I: return "make_double2(-" + a + ".y, " + a + ".x)";
            case S_MI: return "make_double2(" + a + ".y, -" + a + ".x)";
            case S_T:
                return "make_double2((" + a + ".x - " + a + ".y) * " + lit(c) + ", (" + a + ".x + " + a +
                       ".y) * " + lit(c) + ")";
            case S_TDG:
                return "make_double2((" + a + ".x + " + a + ".y) * " + lit(c) + ", (-" + a + ".x + " + a +
                       ".y) * " + lit(c) + ")";
            default: return scale(t.m[2], t.m[3], a);
        }
    }
    std::string diag0(const TileOp& t, const std::string& a) { return scale(t.m[0], t.m[1], a); }
    // (mr + i mi) * a; a real factor (the density-matrix channels' scales) as two multiplies
    // instead of a complex product whose zero imaginary part the compiler cannot drop (IEEE)
    static std::string scale(double mr, double mi, const std::string& a) {
        if (mi != 0.0) return "qcm(" + lit(mr) + ", " + lit(mi) + ", " + a + ")";
        if (mr == 1.0) return a;
        if (mr == -1.0) return "make_double2(-" + a + ".x, -" + a + ".y)";
        return "make_double2(" + lit(mr) + " * " + a + ".x, " + lit(mr) + " * " + a + ".y)";
    }

    void op(const TileOp& t) {
        if (t.cm_out) {  // tile-constant controls: one uniform branch on the tile's load base
            o << "  if ((base & " << hexu(t.cm_out) << ") == " << hexu(t.cm_out) << ") {\n";
            const bool prev = no_rename;
            no_rename = true;  // (register names must agree on both paths)
            op_body(t);
            no_rename = prev;
            o << "  }\n";
            return;
        }
        op_body(t);
    }
    // CX(c -> r) · diag(1, g) on r · CX(c -> r) with g real: each amplitude whose r and c bits
    // differ is scaled by g (the density-matrix depolarizing / phase-damping / phase-flip
    // lowering, density.hip dm_channel).  Emitted as that scale alone — with a thread-bit or
    // tile-constant control the two CXs would otherwise be 2 x 16 predicated selects — and the same
    // products as the three ops (x * 1.0 == x), so bit-identical to them.
    bool xor_diag(const TileOp& a, const TileOp& b, const TileOp& c) {
        auto one_bit = [](uint64_t m) { return m && !(m & (m - 1)); };
        const int nc = (a.cm_reg != 0) + (a.cm_thr != 0) + (a.cm_out != 0);
        if (a.kind != K_M1 || a.sub != S_X || a.p0 < 0 || nc != 1 ||
            !one_bit(a.cm_reg | a.cm_thr | a.cm_out))
            return false;
        if (c.kind != a.kind || c.sub != a.sub || c.p0 != a.p0 || c.cm_reg != a.cm_reg || c.cm_thr != a.cm_thr ||
            c.cm_out != a.cm_out)
            return false;
        if (b.kind != K_DIAG || b.sub != S_GEN || b.p0 != a.p0 || !b.d0_one || b.m[3] != 0.0 || b.cm_reg ||
            b.cm_thr || b.cm_out)
            return false;
        const int P = a.p0;
        const std::string g = lit(b.m[2]);
        if (a.cm_reg) {  // both bits in registers: decided per register here
            const int C = __builtin_ctz(a.cm_reg);
            for (int r = 0; r < R; ++r)
                if (((r >> P) ^ (r >> C)) & 1) o << "  " << v(r) << " = " << scale(b.m[2], 0.0, v(r)) << ";\n";
            return true;
        }
        const std::string pc = "c" + std::to_string(tmp++), f0 = "f" + std::to_string(tmp++),
                          f1 = "f" + std::to_string(tmp++);
        if (a.cm_thr) o << "  const bool " << pc << " = (jb & " << a.cm_thr << "u) != 0u;\n";
        else o << "  const bool " << pc << " = (base & " << hexu(a.cm_out) << ") != 0ull;\n";
        o << "  const double " << f0 << " = " << pc << " ? " << g << " : 1.0, " << f1 << " = " << pc << " ? 1.0 : " << g
          << ";\n";
        for (int r = 0; r < R; ++r) {
            const std::string f = ((r >> P) & 1) ? f1 : f0, x = v(r);
            o << "  " << x << " = make_double2(" << f << " * " << x << ".x, " << f << " * " << x << ".y);\n";
        }
        return true;
    }
    bool no_rename = false;
    void op_body(const TileOp& t) {
        const uint32_t cr = t.cm_reg;
        std::string pred;  // per-thread control predicate (thread-bit controls)
        if (t.cm_thr) {
            pred = "c" + std::to_string(tmp++);
            o << "  const bool " << pred << " = (jb & " << t.cm_thr << "u) == " << t.cm_thr << "u;\n";
        }
        if (t.kind == K_DIAG) {
            std::string tb;
            if (t.p0 < 0) {
                tb = "b" + std::to_string(tmp++);
                o << "  const bool " << tb << " = ((jb >> " << t.b0 << ") & 1u) != 0u;\n";
            }
            for (int r = 0; r < R; ++r) {
                if ((r & cr) != cr) continue;
                const std::string a = v(r);
                std::string nv;
                if (t.p0 >= 0) {
                    const bool bit = (r >> t.p0) & 1;
                    if (!bit && t.d0_one) continue;
                    nv = bit ? diag1(t, a) : diag0(t, a);
                } else {
                    nv = "qsel(" + tb + ", " + diag1(t, a) + ", " + (t.d0_one ? a : diag0(t, a)) + ")";
                }
                if (!pred.empty()) nv = "qsel(" + pred + ", " + nv + ", " + a + ")";
                o << "  " << a << " = " << nv << ";\n";
            }
            return;
        }
        // K_M1 on register bit P (SWAPs were lowered to controlled X by the planner)
        const int P = t.p0;
        for (int r = 0; r < R; ++r) {
            if ((r >> P) & 1) continue;
            if ((r & cr) != cr) continue;  // register-bit controls: decided here, not on the GPU
            const int r1 = r | (1 << P);
            if (t.sub == S_X && pred.empty() && !no_rename) {  // a relabel: no instruction at all
                std::swap(nm[r], nm[r1]);
                continue;
            }
            const std::string a0 = v(r), a1 = v(r1);
            std::string x0, x1;
            switch (t.sub) {
                case S_X: x0 = "t1"; x1 = "t0"; break;
                case S_Y:
                    x0 = "make_double2(t1.y, -t1.x)";
                    x1 = "make_double2(-t0.y, t0.x)";
                    break;
                case S_H:  // unnormalised butterfly; the pass scale restores (1/sqrt2)^k
                    x0 = "make_double2(t0.x + t1.x, t0.y + t1.y)";
                    x1 = "make_double2(t0.x - t1.x, t0.y - t1.y)";
                    break;
                default: break;  // S_GEN: below
            }
            const bool real = t.m[1] == 0.0 && t.m[3] == 0.0 && t.m[5] == 0.0 && t.m[7] == 0.0;
            if (t.sub == S_GEN && real) {  // a real 2x2 (density-matrix bit flip / damping): 4 FMA-able terms
                auto lin = [&](int i, int j) {
                    const std::string ma = lit(t.m[2 * i]), mb = lit(t.m[2 * j]);
                    return "make_double2(" + ma + " * t0.x + " + mb + " * t1.x, " + ma + " * t0.y + " + mb + " * t1.y)";
                };
                o << "  { const double2 t0 = " << a0 << ", t1 = " << a1 << ";\n";
                x0 = lin(0, 1);
                x1 = lin(2, 3);
            } else if (t.sub == S_GEN) {  // double2 has no operator+ here: expand the sums
                auto sum = [](const std::string& a, const std::string& b) {
                    return "make_double2(" + a + ".x + " + b + ".x, " + a + ".y + " + b + ".y)";
                };
                auto cm = [&](int i, const char* a) {
                    return "qcm(" + lit(t.m[2 * i]) + ", " + lit(t.m[2 * i + 1]) + ", " + a + ")";
                };
                o << "  { const double2 t0 = " << a0 << ", t1 = " << a1 << ";\n"
                  << "    const double2 u0 = " << cm(0, "t0") << ", u1 = " << cm(1, "t1") << ";\n"
                  << "    const double2 w0 = " << cm(2, "t0") << ", w1 = " << cm(3, "t1") << ";\n";
                x0 = sum("u0", "u1");
                x1 = sum("w0", "w1");
            } else if (t.sub != S_GEN) {
                o << "  { const double2 t0 = " << a0 << ", t1 = " << a1 << ";\n";
            }
            if (!pred.empty()) {
                x0 = "qsel(" + pred + ", " + x0 + ", t0)";
                x1 = "qsel(" + pred + ", " + x1 + ", t1)";
            }
            o << "    " << a0 << " = " << x0 << ";\n    " << a1 << " = " << x1 << "; }\n";
        }
    }
};

}  // namespace
// Multi-stage passes as persistent, software-pipelined kernels (QSIM_JIT_PIPE: 0 never, 1 for
// 13-qubit tiles only (default), 2 for every multi-stage pass).  Decided from the pass alone, so
// the generator and the launch (grid = resident workgroups) agree.
bool jit_pass_pipelined(const FusedPass& p) {
    static const int v = env_or("QSIM_JIT_PIPE", 1);
    if (p.single >= 0 || p.stage_end - p.stage_begin < 2) return false;
    if (p.relayout) return false;  // (the generator has no pipelined relayout store)
    return v >= 2 || (v == 1 && p.h >= 7);
}
namespace {
// sum_i ((src >> i) & 1) << dst[i] over i < cnt, consecutive bit runs moved by one mask + shift
std::string scatter_expr(const std::string& src, const int* dst, int cnt, bool wide) {
    const std::string ty = wide ? "(unsigned long long)" : "";
    std::string e;
    for (int i = 0; i < cnt;) {
        int k = 1;
        while (i + k < cnt && dst[i + k] == dst[i] + k) ++k;
        const uint64_t m = ((1ull << k) - 1ull) << i;
        std::string t = "(" + ty + "(" + src + " & " + (wide ? hexu(m) : std::to_string((uint32_t)m) + "u") + ")";
        const int sh = dst[i] - i;
        if (sh > 0) t += " << " + std::to_string(sh);
        else if (sh < 0) t += " >> " + std::to_string(-sh);
        t += ")";
        e += e.empty() ? t : " | " + t;
        i += k;
    }
    return e.empty() ? (wide ? std::string("0ull") : std::string("0u")) : e;
}
// OR over i of bit src_pos[i] of `src` moved to bit dst_pos[i] (64-bit), runs of consecutive
// positions (on both sides) moved by one mask + shift
std::string gather_scatter_expr(const std::string& src, const int* src_pos, const int* dst_pos, int cnt) {
    std::string e;
    for (int i = 0; i < cnt;) {
        int k = 1;
        while (i + k < cnt && src_pos[i + k] == src_pos[i] + k && dst_pos[i + k] == dst_pos[i] + k) ++k;
        const uint64_t m = ((1ull << k) - 1ull) << src_pos[i];
        std::string t = "((" + src + " & " + hexu(m) + ")";
        const int sh = dst_pos[i] - src_pos[i];
        if (sh > 0) t += " << " + std::to_string(sh);
        else if (sh < 0) t += " >> " + std::to_string(-sh);
        t += ")";
        e += e.empty() ? t : " | " + t;
        i += k;
    }
    return e.empty() ? std::string("0ull") : e;
}
// Thread index spread over the tile bits that are not register bits of stage `st`.
std::string jb_expr(const Stage& st, int rb, int tile_bits) {
    if (st.tscatter) return scatter_expr("tid", st.tmap, tile_bits - rb, false);
    std::string e = "tid";
    for (int i = 0; i < rb; ++i) e = "qins0(" + e + ", " + std::to_string(st.fix[i]) + ")";
    return e;
}

// Workgroup -> tile order (workgroups are dispatched round-robin over the 8 XCDs, so the low 3
// bits of blockIdx pick the XCD).  QSIM_JIT_XCD: 0 natural (consecutive workgroups take
// consecutive tiles); 1 each XCD streams one contiguous eighth of the tiles; s >= 2: the XCD bits
// move to tile-id bits s-2 .. s (XCDs interleave at that granularity); -1 bit-reversed ids.
int jit_xcd() {
    static const int v = env_or("QSIM_JIT_XCD", 1);
    return v;
}
// CX · real diag · CX triples emitted as one scale (Gen::xor_diag; QSIM_JIT_XOR_DIAG=0: as three ops)
bool xor_diag_on() {
    static const bool v = env_or("QSIM_JIT_XOR_DIAG", 1) != 0;
    return v;
}
std::string tile_id_expr() {
    const int x = jit_xcd();
    const std::string b = "(unsigned long long)blockIdx.x";
    if (x == 1)
        return "  const unsigned long long tile_id = (gridDim.x & 7u) ? " + b + " : (" + b +
               " & 7ull) * (gridDim.x >> 3) + (" + b + " >> 3);\n";
    if (x >= 2) {
        const int s = x - 2;  // XCD bits land at tile-id bits s..s+2
        const std::string lo = "((" + b + " >> 3) & " + hexu((1ull << s) - 1ull) + ")";
        const std::string hi = "((" + b + " >> " + std::to_string(3 + s) + ") << " + std::to_string(s + 3) + ")";
        return "  const unsigned long long tile_id = (gridDim.x & " + std::to_string((8u << s) - 1u) + "u) ? " + b +
               " : (" + hi + " | ((" + b + " & 7ull) << " + std::to_string(s) + ") | " + lo + ");\n";
    }
    if (x == -1)
        return "  const unsigned long long tile_id = (gridDim.x & (gridDim.x - 1u)) ? " + b +
               " : (unsigned long long)(__builtin_bitreverse32(blockIdx.x) >> (32 - (31 - __builtin_clz(gridDim.x))));\n";
    return "  const unsigned long long tile_id = blockIdx.x;\n";
}

void gen_pass(std::ostringstream& out, const Plan& plan, const FusedPass& p, int idx) {
    const int H = p.h, RB = p.rb, R = 1 << RB, T = 64 << H;
    const int r0 = p.r0, nh = 6 + H - r0;
    const bool pipe = jit_pass_pipelined(p);
    if (pipe && p.relayout) fail(QSIM_ERR_RUNTIME, "relayout passes are not pipelined");
    Gen g;
    g.R = R;
    g.RB = RB;
    for (int r = 0; r < R; ++r) g.nm[r] = r;
    std::ostringstream& o = g.o;
    // zmask: positions the tile-id bits skip — the tile's own qubits above the run, plus (for a
    // sub-space launch of the sharded engine) fixed qubits whose values fix_val supplies.  Zero
    // insertion in ascending position order, uniform per workgroup (scalar ALU).
    auto tile_base = [&](const std::string& tid_var, const std::string& base_var) {
        o << "  { unsigned long long k = (" << tid_var << " & tpt_mask) << " << r0 << ";\n"
          << "    for (unsigned long long m = zmask; m; m &= m - 1ull) {\n"
          << "      const unsigned long long lo = k & ((1ull << __builtin_ctzll(m)) - 1ull);\n"
          << "      k = ((k ^ lo) << 1) | lo;\n    }\n"
          << "    " << base_var << " = (" << tid_var << " >> log_tpt) * stride + (k | fix_val); }\n";
    };
    // thread part of a stage's HBM address (the tile base is OR-ed in)
    auto gthread = [&](const Stage& st) {
        std::string e = "(unsigned long long)(jb & " + std::to_string((1u << r0) - 1u) + "u)";
        for (int i = 0; i < nh; ++i)
            e += " | ((unsigned long long)((jb >> " + std::to_string(r0 + i) + ") & 1u) << " +
                 std::to_string(p.hpos[i]) + ")";
        (void)st;
        return e;
    };
    o << "extern \"C\" __global__ void __launch_bounds__(" << (T >> RB) << ", " << (H >= 7 ? 1 : 2)
      << ")\nqk" << idx
      << "(double2* __restrict__ st, unsigned long long stride, unsigned long long tpt_mask, int log_tpt,"
         " unsigned long long zmask, unsigned long long fix_val, unsigned long long ntiles"
      << (p.relayout ? ", double2* __restrict__ dst" : "") << ") {\n"
      << "  __shared__ double2 tile[" << T << "];\n"
      << "  char* const lds = reinterpret_cast<char*>(tile);\n"
      << "  const unsigned tid = threadIdx.x;\n";
    o << "  double2";
    for (int r = 0; r < R; ++r) o << (r ? ", v" : " v") << r;
    o << ";\n";
    const int sb = p.stage_begin, se = p.stage_end;
    if (pipe) {
        // Persistent, software-pipelined: each workgroup walks tiles it = 0, 1, ... of its share
        // (each XCD streams one contiguous eighth when the counts allow); the HBM loads of the
        // next tile are issued right after the first stage's LDS write, so they are in flight
        // during the LDS stages and the stores of the current tile (one big-LDS workgroup per CU
        // otherwise leaves HBM idle between its load and store phases).
        o << "  double2";
        for (int r = 0; r < R; ++r) o << (r ? ", w" : " w") << r;
        o << ";\n"
          << "  const unsigned long long G = gridDim.x, b = blockIdx.x;\n"
          << "  const bool xo = ((ntiles & 7ull) == 0ull) && ((G & 7ull) == 0ull);\n"
          << "  const unsigned long long per = ntiles >> 3, gx = G >> 3;\n"
          << "  unsigned long long it = 0;\n"
          ;
        if (env_or("QSIM_JIT_PIPE_ORDER", 1) == 1)  // each workgroup streams one contiguous range (default)
            o << "  const bool cw = (ntiles % G) == 0ull;\n  const unsigned long long tpw = ntiles / G;\n"
              << "  auto tile_at = [&](unsigned long long i) { return cw ? b * tpw + i : i * G + b; };\n"
              << "  auto tile_ok = [&](unsigned long long i) { return cw ? i < tpw : (i * G + b < ntiles); };\n";
        else
            o << "  auto tile_at = [&](unsigned long long i) { return xo ? (b & 7ull) * per + i * gx + (b >> 3) : i * G + b; };\n"
              << "  auto tile_ok = [&](unsigned long long i) { return xo ? (i * gx + (b >> 3) < per) : (i * G + b < ntiles); };\n";
        o
          << "  if (!tile_ok(0)) return;\n"
          << "  unsigned long long base, nbase = 0;\n"
          << "  { const unsigned long long t0 = tile_at(0);\n";
        tile_base("t0", "base");
        o << "  }\n";
        {
            const Stage& st0 = plan.stages[sb];
            o << "  const unsigned long long gth0 = [&] { const unsigned jb = " << jb_expr(st0, RB, 6 + H) << "; return "
              << gthread(st0) << "; }();\n";
            for (int r = 0; r < R; ++r) o << "  v" << r << " = qld(st + (base | gth0 | " << hexu(st0.goff[r]) << "));\n";
        }
        // the tile body is emitted twice: a peeled first tile, then the loop, so the loop head is
        // reached only with the previous tile's stores outstanding behind the prefetch (a single
        // loop merges that state with the prologue's and waits for the stores too)
    } else {
        o << tile_id_expr() << "  unsigned long long base;\n";
        tile_base("tile_id", "base");
        if (p.relayout) {  // the tile's base under the store layout: every non-tile load
                           // position's bit (tile-id and a sub-space launch's fixed bits) moved
            int nt_pos[32], k = 0;
            uint64_t hm = 0;
            for (int i = 0; i < nh; ++i) hm |= 1ull << p.hpos[i];
            for (int q = r0; k < p.n_tid && q < 64; ++q)
                if (!((hm >> q) & 1ull)) nt_pos[k++] = q;
            o << "  const unsigned long long bl = base - (tile_id >> log_tpt) * stride;\n"
              << "  const unsigned long long base_st = (tile_id >> log_tpt) * stride | ("
              << gather_scatter_expr("bl", nt_pos, p.st_tid, p.n_tid) << ");\n";
        }
    }
    auto body = [&]() {
        for (int r = 0; r < R; ++r) g.nm[r] = r;
        if (pipe) o << "  const bool more = tile_ok(it + 1);\n";
        for (int s = sb; s < se; ++s) {
            const Stage& st = plan.stages[s];
            o << "  {\n  const unsigned jb = " << jb_expr(st, RB, 6 + H) << ";\n";
            if (s == sb && pipe) o << "  const unsigned long long gb = base | gth0;\n";
            else if (s == se - 1 && p.relayout) {
                int dst[16];
                for (int i = 0; i < 6 + H - RB; ++i) dst[i] = p.st_pos[st.tmap[i]];
                o << "  const unsigned long long gb = base_st | " << scatter_expr("(unsigned long long)tid", dst, 6 + H - RB, true) << ";\n";
            } else if (s == sb || s == se - 1) o << "  const unsigned long long gb = base | " << gthread(st) << ";\n";
            auto sigma_expr = [](const uint32_t* trow) {
                std::string e = "jb";
                for (int i = 0; i < 4; ++i)
                    e += " ^ ((__builtin_popcount(jb & " + std::to_string(trow[i]) + "u) & 1u) << " +
                         std::to_string(i) + ")";
                return e;
            };
            if (s != sb) o << "  const unsigned lb = 16u * (" << sigma_expr(st.trow_in) << ");\n";
            if (s != se - 1) o << "  const unsigned lbw = 16u * (" << sigma_expr(st.trow_out) << ");\n";
            if (s == sb) {
                if (!pipe)
                    for (int r = 0; r < R; ++r) o << "  " << g.v(r) << " = qld(st + (gb | " << hexu(st.goff[r]) << "));\n";
            } else {
                for (int r = 0; r < R; ++r)
                    o << "  " << g.v(r) << " = *reinterpret_cast<const double2*>(lds + (lb ^ " << st.lds[r] << "u));\n";
            }
            for (int i = st.op_begin; i < st.op_end; ++i) {
                if (xor_diag_on() && i + 2 < st.op_end && g.xor_diag(plan.ops[i], plan.ops[i + 1], plan.ops[i + 2])) {
                    i += 2;
                    continue;
                }
                g.op(plan.ops[i]);
            }
            if (s == se - 1) {
                const double sc = std::ldexp(1.0, -(p.hu_count / 2)) * ((p.hu_count & 1) ? kInvSqrt2 : 1.0);
                for (int r = 0; r < R; ++r) {
                    std::string val = g.v(r);
                    if (sc != 1.0) val = "make_double2(" + val + ".x * " + lit(sc) + ", " + val + ".y * " + lit(sc) + ")";
                    o << "  qst(" << (p.relayout ? "dst" : "st") << " + (gb | " << hexu(st.goff[r]) << "), " << val << ");\n";
                }
            } else {
                for (int r = 0; r < R; ++r)
                    o << "  *reinterpret_cast<double2*>(lds + (lbw ^ " << st.lds_w[r] << "u)) = " << g.v(r) << ";\n";
                o << "  __syncthreads();\n";
                if (pipe && s == sb) {  // prefetch the next tile's first-stage registers (the last
                                        // tile re-reads itself: no branch around the loads)
                    o << "  {\n    const unsigned long long tn = tile_at(more ? it + 1 : it);\n";
                    tile_base("tn", "nbase");
                    for (int r = 0; r < R; ++r)
                        o << "    w" << r << " = qld(st + (nbase | gth0 | " << hexu(plan.stages[sb].goff[r]) << "));\n";
                    o << "  }\n";
                }
            }
            o << "  }\n";
        }
        if (pipe) {
            o << "  if (!more) return;\n  __syncthreads();  // the last stage's LDS reads precede the next tile's writes\n"
              << "  base = nbase;\n  ++it;\n";
            for (int r = 0; r < R; ++r) o << "  v" << r << " = w" << r << ";\n";
        }
    };
    if (pipe) {
        body();
        o << "  for (;;) {\n";
        body();
        o << "  }\n";
    } else {
        body();
    }
    o << "}\n";
    out << o.str();
}

}  // namespace

// Passes with very many ops stay on the interpreter: straight-line code grows with every op
// (each expanded over its register pairs) and hipRTC time with it; past ~kJitMaxOps ops the
// pass is VALU-heavy anyway and the per-op dispatch of the interpreter matters less.
constexpr int kJitMaxOps = 192;
static int pass_ops(const Plan& plan, const FusedPass& p) {
    int ops = 0;
    for (int k = p.stage_begin; k < p.stage_end; ++k) ops += plan.stages[k].op_end - plan.stages[k].op_begin;
    return ops;
}
static bool jit_pass_eligible(const Plan& plan, const FusedPass& p) {
    return p.single < 0 && p.h >= 4 && pass_ops(plan, p) <= kJitMaxOps;
}
// The passes one code object specialises: eligible passes in plan order while the module stays
// within kJitModuleOps ops (bounds hipRTC time — also for the background worker, which a
// process exit waits for); later passes run on the interpreter.
constexpr int kJitModuleOps = 2048;
static std::vector<char> jit_selection(const Plan& plan) {
    std::vector<char> sel(plan.passes.size(), 0);
    int budget = kJitModuleOps;
    for (size_t i = 0; i < plan.passes.size(); ++i) {
        if (!jit_pass_eligible(plan, plan.passes[i])) continue;
        const int ops = pass_ops(plan, plan.passes[i]);
        if (ops > budget) break;
        budget -= ops;
        sel[i] = 1;
    }
    return sel;
}

std::string jit_source(const Plan& plan) {
    std::ostringstream out;
    bool any = false;
    out << (env_or("QSIM_JIT_NT", 1) ? kPreludeNT : kPreludeT) << kPrelude;
    const std::vector<char> sel = jit_selection(plan);
    for (size_t i = 0; i < plan.passes.size(); ++i) {
        if (!sel[i]) continue;
        gen_pass(out, plan, plan.passes[i], (int)i);
        any = true;
    }
    return any ? out.str() : std::string();
}

// ---------------------------------------------------------------------------------------
// Compilation (hipRTC) on one background worker
// ---------------------------------------------------------------------------------------
struct JitJob {
    std::string src;
    std::vector<char> code;
    std::string log;
    std::atomic<int> state{0};  // 0 queued, 1 done ok, 2 failed
};

bool jit_compile(const std::string& src, std::vector<char>& code, std::string& log) {
    if (const char* dir = std::getenv("QSIM_JIT_DUMP")) {  // keep every generated source (debugging)
        static std::atomic<int> seq{0};
        const std::string path = std::string(dir) + "/qsim_jit_" + std::to_string(seq++) + ".hip";
        if (FILE* f = std::fopen(path.c_str(), "w")) {
            std::fwrite(src.data(), 1, src.size(), f);
            std::fclose(f);
        }
    }
    const char* opts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17"};
    // the code object of this source from the on-disk cache (cache.hip), when a process on this
    // machine compiled it before
    int vmaj = 0, vmin = 0;
    (void)hiprtcVersion(&vmaj, &vmin);
    const std::string okey = std::string(opts[0]) + " " + opts[1] + " " + opts[2] + " hiprtc " +
                             std::to_string(vmaj) + "." + std::to_string(vmin);
    if (jit_cache_load(src, okey, code)) return true;
    hiprtcProgram prog;
    if (hiprtcCreateProgram(&prog, src.c_str(), "qsim_pass.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS) {
        log = "hiprtcCreateProgram failed";
        return false;
    }
    const hiprtcResult rc = hiprtcCompileProgram(prog, 3, opts);
    size_t ls = 0;
    hiprtcGetProgramLogSize(prog, &ls);
    if (ls > 1) {
        log.resize(ls);
        hiprtcGetProgramLog(prog, &log[0]);
    }
    bool ok = rc == HIPRTC_SUCCESS;
    if (ok) {
        size_t cs = 0;
        hiprtcGetCodeSize(prog, &cs);
        code.resize(cs);
        ok = cs > 0 && hiprtcGetCode(prog, code.data()) == HIPRTC_SUCCESS;
    }
    hiprtcDestroyProgram(&prog);
    if (ok) jit_cache_store(src, okey, code);
    return ok;
}

namespace {
class Worker {
public:
    static Worker& get() {
        static Worker w;
        return w;
    }
    void submit(std::shared_ptr<JitJob> j) {
        {
            std::lock_guard<std::mutex> l(mu_);
            if (stop_) {  // shut down (process exit): the plan stays on the interpreter
                j->log = "JIT worker stopped";
                j->state.store(2);
                return;
            }
            q_.push_back(std::move(j));
            if (!th_.joinable()) th_ = std::thread([this] { loop(); });
        }
        cv_.notify_one();
    }
    // Drop queued jobs and wait for the compile in progress.  Must run before the compiler's own
    // static state is torn down at exit: a compile still running while LLVM's statics are
    // destroyed dies with "LLVM ERROR" (seen in a pytest process that exited mid-compile).
    void shutdown() {
        {
            std::lock_guard<std::mutex> l(mu_);
            stop_ = true;
            for (auto& j : q_) {
                j->log = "JIT worker stopped";
                j->state.store(2);
            }
            q_.clear();
        }
        cv_.notify_all();
        std::lock_guard<std::mutex> l(join_mu_);
        if (th_.joinable() && th_.get_id() != std::this_thread::get_id()) th_.join();
    }
    ~Worker() { shutdown(); }

private:
    void loop() {
        for (;;) {
            std::shared_ptr<JitJob> j;
            {
                std::unique_lock<std::mutex> l(mu_);
                cv_.wait(l, [&] { return stop_ || !q_.empty(); });
                if (stop_) return;
                j = q_.front();
                q_.pop_front();
            }
            const bool ok = jit_compile(j->src, j->code, j->log);
            j->state.store(ok ? 1 : 2);
            // The first compile constructed the compiler's static objects; an exit handler
            // registered after them runs before their destructors (reverse registration order).
            if (!atexit_registered_) {
                atexit_registered_ = true;
                std::atexit([] { Worker::get().shutdown(); });
            }
        }
    }
    std::mutex mu_, join_mu_;
    bool atexit_registered_ = false;
    std::condition_variable cv_;
    std::deque<std::shared_ptr<JitJob>> q_;
    std::thread th_;
    bool stop_ = false;
};
}  // namespace

void jit_shutdown() { Worker::get().shutdown(); }

JitModule::~JitModule() {
    // the owner has drained the stream that ran this module's kernels (engine destructors
    // synchronise first; PlanCache::get synchronises before it evicts a plan)
    if (mod) (void)hipModuleUnload(mod);
}

const JitModule* jit_for(JitState& js, const Plan& plan, int n) {
    const int mode = jit_mode();
    if (mode == 0 || n < jit_min_qubits() || js.failed) return nullptr;
    if (js.mod) return js.mod.get();
    if (!js.job) {
        std::string src = jit_source(plan);
        if (src.empty()) {
            js.failed = true;  // nothing to specialise (no staged pass)
            return nullptr;
        }
        js.job = std::make_shared<JitJob>();
        js.job->src = std::move(src);
        if (mode == 2) {
            const bool ok = jit_compile(js.job->src, js.job->code, js.job->log);
            js.job->state.store(ok ? 1 : 2);
        } else {
            Worker::get().submit(js.job);
        }
    }
    const int st = js.job->state.load();
    if (st == 0) return nullptr;  // still compiling: the interpreter runs this time
    if (st == 2) {
        js.failed = true;
        std::fprintf(stderr, "qsim: pass JIT failed, staying on the interpreter:\n%s\n", js.job->log.c_str());
        js.job.reset();
        return nullptr;
    }
    auto m = std::make_unique<JitModule>();
    QSIM_HIPCHK(hipModuleLoadData(&m->mod, js.job->code.data()));
    m->fn.assign(plan.passes.size(), nullptr);
    const std::vector<char> sel = jit_selection(plan);
    for (size_t i = 0; i < plan.passes.size(); ++i) {
        if (!sel[i]) continue;
        const std::string name = "qk" + std::to_string(i);
        QSIM_HIPCHK(hipModuleGetFunction(&m->fn[i], m->mod, name.c_str()));
    }
    js.job.reset();
    js.mod = std::move(m);
    return js.mod.get();
}

}  // namespace qsim_hip
