// density.hip — DensityMatrix / DensityMatrixSimulator (reference include/DensityMatrix.cuh:63-224,
// src/DensityMatrix.cu) on the state-vector engine.
//
// Layout: rho (2^n x 2^n, row-major like the reference, src/DensityMatrix.cu:29-30) is the vector
// of a qsim_state with 2n index bits, v[i * 2^n + j] = rho[i][j]: bits 0..n-1 are the column j,
// bits n..2n-1 the row i.  U rho U^dag is U on row bit q+n and conj(U) on column bit q — two
// ordinary engine ops — and every channel of the reference is a short sequence of controlled 2x2 /
// diagonal ops on the bit pair (r = q+n, c = q): CNOT(c -> r) maps the element pairs
// (rho_rc, rho_r'c') (r' = 1-r, c' = 1-c) onto pairs along c and marks the off-diagonal elements
// by r ^ c.  A density-matrix circuit is therefore an op list for the same fused LDS tile passes,
// circuit-specialised kernels and per-gate kernels as a 2n-qubit state (no 4^n-thread kernels);
// 4^15 x 16 B = 16 GiB fits one MI355X (the reference stops at 14, :25-27).
//
// Reference semantics kept: gates X..Rz, CNOT, CZ, SWAP (others throw runtime_error, :264-266);
// after each gate, for each of its qubits, every channel that applies to the qubit (empty qubit
// list = all, :201-212, :269-296); depolarizing scales the off-diagonal by 1 - 4p/3 and leaves the
// diagonal (:978-1002); amplitude damping rho00 += g rho11, rho11 *= 1 - g, off-diagonal *=
// sqrt(1 - g) (:1004-1044; the reference reads rho11 racily, here the pre-channel value); phase
// damping / phase flip scale the off-diagonal by sqrt(1 - g) / 1 - 2p (:1046-1065, :1102-1122); bit
// flip mixes rho_rc with rho_r'c' (:1067-1100); bit-phase flip is the phase-flip channel
// (:343-356).  Divergence: Y acts as Y rho Y^dag; the reference kernel's phase table (:540-544)
// returns -(Y rho Y^dag) (trace -1; untested there).
#include <hip/hip_runtime.h>

#include <cmath>
#include <string>
#include <vector>

#include "engine.hpp"
#include "qsim_hip.h"

namespace qsim_hip {

static Op dm_row(Op o, int n) {  // the op on the row bits
    o.t0 += n;
    if (o.t1 >= 0) o.t1 += n;
    o.cmask <<= n;
    return o;
}
static Op dm_col(Op o) {  // conj(op) on the column bits
    for (int i = 1; i < 8; i += 2) o.m[i] = -o.m[i];
    if (o.kind == K_M1 && o.sub == S_Y) o.sub = S_GEN;  // conj(Y) = [[0, i], [-i, 0]]
    if (o.kind == K_DIAG) {
        if (o.sub == S_I) o.sub = S_MI;
        else if (o.sub == S_MI) o.sub = S_I;
        else if (o.sub == S_T) o.sub = S_TDG;
        else if (o.sub == S_TDG) o.sub = S_T;
    }
    return o;
}

static void dm_channel(std::vector<Op>& out, int n, int type, int q, double p) {
    const int r = q + n, c = q;
    auto m1 = [&](int t, uint64_t cm, double a, double b, double cc, double d, int sub = S_GEN) {
        Op o;
        o.kind = K_M1;
        o.sub = sub;
        o.t0 = t;
        o.cmask = cm;
        const double v[8] = {a, 0, b, 0, cc, 0, d, 0};
        for (int i = 0; i < 8; ++i) o.m[i] = v[i];
        out.push_back(o);
    };
    auto cx = [&]() { m1(r, 1ull << c, 0, 1, 1, 0, S_X); };
    auto diag = [&](double d0, double d1) {
        Op o;
        o.kind = K_DIAG;
        o.sub = S_GEN;
        o.t0 = r;
        o.d0_one = d0 == 1.0;
        o.m[0] = d0;
        o.m[2] = d1;
        out.push_back(o);
    };
    switch (type) {
        case 0: cx(); diag(1.0, 1.0 - 4.0 * p / 3.0); cx(); break;          // depolarizing (ref.)
        case 1:                                                              // amplitude damping
            cx();
            m1(r, 0, 0, 1, 1, 0, S_X);                   // r' = r ^ c ^ 1: 1 on the diagonal block
            m1(c, 1ull << r, 1.0, p, 0.0, 1.0 - p);      // [rho00, rho11] <- [[1, g], [0, 1-g]]
            diag(std::sqrt(1.0 - p), 1.0);               // off-diagonal elements
            m1(r, 0, 0, 1, 1, 0, S_X);
            cx();
            break;
        case 2: cx(); diag(1.0, std::sqrt(1.0 - p)); cx(); break;           // phase damping
        case 3: cx(); m1(c, 0, 1.0 - p, p, p, 1.0 - p); cx(); break;        // bit flip
        case 4: case 5: cx(); diag(1.0, 1.0 - 2.0 * p); cx(); break;       // phase / bit-phase flip
        default: fail(QSIM_ERR_INVALID_ARGUMENT, "unknown noise type");
    }
}

void dm_lower(int n, const qsim_gate* gates, size_t count, const qsim_noise_channel* ch,
              size_t nch, std::vector<Op>& out, bool reference_y) {
    for (size_t c = 0; c < nch; ++c) {
        if (ch[c].type < 0 || ch[c].type > 5) fail(QSIM_ERR_INVALID_ARGUMENT, "unknown noise type");
        if (ch[c].qubit < -1 || ch[c].qubit >= n)
            fail(QSIM_ERR_OUT_OF_RANGE, "Qubit index " + std::to_string(ch[c].qubit) + " out of range");
    }
    for (size_t i = 0; i < count; ++i) {
        const qsim_gate& g = gates[i];
        if (g.type == QSIM_GATE_CRY || g.type == QSIM_GATE_CRZ || g.type == QSIM_GATE_TOFFOLI)
            fail(QSIM_ERR_RUNTIME, "Gate not supported in density matrix simulation");
        Op o = lower_gate(g, n);
        o.src = (int)i;
        out.push_back(dm_row(o, n));
        out.push_back(dm_col(o));
        if (reference_y && g.type == QSIM_GATE_Y) {  // dmApplyY's extra sign (-Y rho Y^dag)
            Op neg;
            neg.kind = K_DIAG;
            neg.sub = S_GEN;
            neg.t0 = 0;
            neg.d0_one = false;
            neg.m[0] = neg.m[2] = -1.0;
            neg.src = (int)i;
            out.push_back(neg);
        }
        for (int k = 0; k < g.nqubits; ++k)
            for (size_t c = 0; c < nch; ++c)
                if (ch[c].qubit < 0 || ch[c].qubit == g.qubits[k])
                    dm_channel(out, n, ch[c].type, g.qubits[k], ch[c].probability);
    }
}

void dm_lower_channel(int n, int type, int qubit, double p, std::vector<Op>& out) {
    if (qubit < 0 || qubit >= n) fail(QSIM_ERR_OUT_OF_RANGE, "Qubit index " + std::to_string(qubit) + " out of range");
    dm_channel(out, n, type, qubit, p);
}

__global__ __launch_bounds__(256) void k_dm_diag(const double2* rho, uint64_t dim, double* out) {
    const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < dim; i += step)
        out[i] = rho[i * (dim + 1)].x;
}

// rho[i][j] = psi_i conj(psi_j) (dmInitPure, src/DensityMatrix.cu:412-425) or, psi == null, I / dim.
__global__ __launch_bounds__(256) void k_dm_init(double2* rho, const double2* psi, int n) {
    const uint64_t dim = 1ull << n, total = dim << n;
    const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < total; k += step) {
        const uint64_t i = k >> n, j = k & (dim - 1);
        if (psi) {
            const double2 si = psi[i], sj = psi[j];
            rho[k] = make_double2(si.x * sj.x + si.y * sj.y, si.y * sj.x - si.x * sj.y);
        } else {
            rho[k] = make_double2(i == j ? 1.0 / (double)dim : 0.0, 0.0);
        }
    }
}

void launch_dm_diag(const double2* rho, int n, double* out, hipStream_t s) {
    const uint64_t dim = 1ull << n;
    const unsigned blocks = (unsigned)std::min<uint64_t>((dim + 255) / 256, 1024);
    hipLaunchKernelGGL(k_dm_diag, dim3(blocks), dim3(256), 0, s, rho, dim, out);
    QSIM_HIPCHK(hipGetLastError());
}

void launch_dm_init(double2* rho, const double2* psi, int n, hipStream_t s) {
    const uint64_t total = 1ull << (2 * n);
    const unsigned blocks = (unsigned)std::min<uint64_t>((total + 255) / 256, 256 * 32);
    hipLaunchKernelGGL(k_dm_init, dim3(blocks), dim3(256), 0, s, rho, psi, n);
    QSIM_HIPCHK(hipGetLastError());
}

}  // namespace qsim_hip
