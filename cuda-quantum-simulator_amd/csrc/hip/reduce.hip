// reduce.hip — state initialisation and the readout consumers of the hot path: probabilities,
// wave64 norm / single-bit-probability reductions, collapse, device-side sampling and the batch
// average of |a|^2.
//
// Reference behaviour (src/StateVector.cu): initializeZero/Basis :24-39, probabilityKernel
// :41-48, qubitProbabilityKernel + host sum :83-99/:280-287, collapseStateKernel :105-124,
// sample :316-342 (partial_sum CDF + lower_bound), BatchedSimulator::getAverageProbabilities
// src/NoiseModel.cu:894-914.  The reference copies 2^n doubles to the host for every sum; here
// sums are wave64 __shfl_down reductions -> one partial per workgroup -> a single-workgroup
// pass that adds the partials in a fixed order (bitwise reproducible run to run).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "device_ops.hpp"
#include "engine.hpp"

namespace qsim_hip {

constexpr int kReduceBlocks = 2048;

__global__ __launch_bounds__(256) void k_init_basis(double2* st, uint64_t total, uint64_t stride,
                                                    uint64_t basis) {
    const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += step) {
        const bool one = (i & (stride - 1)) == basis;
        st[i] = make_double2(one ? 1.0 : 0.0, 0.0);
    }
}

void launch_init_basis(double2* st, int n, uint64_t batch, uint64_t basis, hipStream_t s) {
    const uint64_t total = batch << n;
    const uint64_t blocks = std::min<uint64_t>((total + 255) / 256, 256 * 32);
    hipLaunchKernelGGL(k_init_basis, dim3((unsigned)blocks), dim3(256), 0, s, st, total,
                       1ull << n, basis);
    QSIM_HIPCHK(hipGetLastError());
}

__global__ __launch_bounds__(256) void k_probabilities(const double2* st, uint64_t count,
                                                       double* out) {
    const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += step) {
        const double2 a = st[i];
        out[i] = a.x * a.x + a.y * a.y;
    }
}

void launch_probabilities(const double2* st, uint64_t count, double* out, hipStream_t s) {
    const uint64_t blocks = std::min<uint64_t>((count + 255) / 256, 256 * 32);
    hipLaunchKernelGGL(k_probabilities, dim3((unsigned)blocks), dim3(256), 0, s, st, count, out);
    QSIM_HIPCHK(hipGetLastError());
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off);
    return v;
}

// Sum |a_i|^2 over the indices enumerated by k in [0, count): i = insert0(k, bit) if bit >= 0
// (only bit==0 amplitudes; for bit >= 6 this halves the bytes read), else i = k.
__global__ __launch_bounds__(256) void k_norm_partial(const double2* st, uint64_t count, int bit,
                                                      double* partials) {
    __shared__ double wsum[4];
    double acc = 0.0;
    const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < count; k += step) {
        uint64_t i = k;
        if (bit >= 0) {
            const uint64_t lo = k & ((1ull << bit) - 1ull);
            i = ((k ^ lo) << 1) | lo;
        }
        const double2 a = st[i];
        acc += a.x * a.x + a.y * a.y;
    }
    acc = wave_sum(acc);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) partials[blockIdx.x] = (wsum[0] + wsum[1]) + (wsum[2] + wsum[3]);
}

__global__ __launch_bounds__(256) void k_sum_partials(const double* partials, int count,
                                                      double* result) {
    __shared__ double wsum[4];
    double acc = 0.0;
    for (int i = threadIdx.x; i < count; i += 256) acc += partials[i];
    acc = wave_sum(acc);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) *result = (wsum[0] + wsum[1]) + (wsum[2] + wsum[3]);
}

double reduce_norm(const double2* st, int n, int bit, double* d_partials, double* d_result,
                   hipStream_t s) {
    const uint64_t count = bit >= 0 ? (1ull << (n - 1)) : (1ull << n);
    const int blocks = (int)std::min<uint64_t>((count + 255) / 256, kReduceBlocks);
    hipLaunchKernelGGL(k_norm_partial, dim3(blocks), dim3(256), 0, s, st, count, bit, d_partials);
    QSIM_HIPCHK(hipGetLastError());
    hipLaunchKernelGGL(k_sum_partials, dim3(1), dim3(256), 0, s, d_partials, blocks, d_result);
    QSIM_HIPCHK(hipGetLastError());
    double h = 0.0;
    QSIM_HIPCHK(hipMemcpyAsync(&h, d_result, sizeof(double), hipMemcpyDeviceToHost, s));
    QSIM_HIPCHK(hipStreamSynchronize(s));
    return h;
}

// max over i of max(|re a_i - re b_i|, |im a_i - im b_i|): the per-component bar of the parity
// tests (reference tests/test_gpu_cpu_equivalence.cu:26), computed where both states live (a
// 30-qubit comparison would otherwise copy 32 GiB to the host).  Max is order-free: deterministic.
__global__ __launch_bounds__(256) void k_maxdiff_partial(const double2* a, const double2* b,
                                                         uint64_t count, double* partials) {
    __shared__ double wmax[4];
    double m = 0.0;
    const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += step) {
        const double2 x = a[i], y = b[i];
        const double d = fmax(fabs(x.x - y.x), fabs(x.y - y.y));
        m = d > m || d != d ? d : m;  // (a NaN difference propagates)
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const double o = __shfl_down(m, off);
        m = o > m || o != o ? o : m;
    }
    if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        double r = wmax[0];
        for (int w = 1; w < 4; ++w) r = wmax[w] > r || wmax[w] != wmax[w] ? wmax[w] : r;
        partials[blockIdx.x] = r;
    }
}

__global__ __launch_bounds__(256) void k_max_partials(const double* partials, int count, double* result) {
    __shared__ double wmax[4];
    double m = 0.0;
    for (int i = threadIdx.x; i < count; i += 256) m = partials[i] > m || partials[i] != partials[i] ? partials[i] : m;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const double o = __shfl_down(m, off);
        m = o > m || o != o ? o : m;
    }
    if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        double r = wmax[0];
        for (int w = 1; w < 4; ++w) r = wmax[w] > r || wmax[w] != wmax[w] ? wmax[w] : r;
        *result = r;
    }
}

double reduce_max_abs_diff(const double2* a, const double2* b, int n, double* d_partials, double* d_result,
                           hipStream_t s) {
    const uint64_t count = 1ull << n;
    const int blocks = (int)std::min<uint64_t>((count + 255) / 256, kReduceBlocks);
    hipLaunchKernelGGL(k_maxdiff_partial, dim3(blocks), dim3(256), 0, s, a, b, count, d_partials);
    QSIM_HIPCHK(hipGetLastError());
    hipLaunchKernelGGL(k_max_partials, dim3(1), dim3(256), 0, s, d_partials, blocks, d_result);
    QSIM_HIPCHK(hipGetLastError());
    double h = 0.0;
    QSIM_HIPCHK(hipMemcpyAsync(&h, d_result, sizeof(double), hipMemcpyDeviceToHost, s));
    QSIM_HIPCHK(hipStreamSynchronize(s));
    return h;
}

__global__ __launch_bounds__(256) void k_collapse(double2* st, uint64_t count, int bit, int result,
                                                  double scale) {
    const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += step) {
        const int v = (int)((i >> bit) & 1ull);
        const double2 a = st[i];
        st[i] = v != result ? make_double2(0.0, 0.0) : make_double2(a.x * scale, a.y * scale);
    }
}

void launch_collapse(double2* st, int n, int bit, int result, double scale, hipStream_t s) {
    const uint64_t count = 1ull << n;
    const uint64_t blocks = std::min<uint64_t>((count + 255) / 256, 256 * 32);
    hipLaunchKernelGGL(k_collapse, dim3((unsigned)blocks), dim3(256), 0, s, st, count, bit, result,
                       scale);
    QSIM_HIPCHK(hipGetLastError());
}

// ---- sampling: chunk sums on device, chunk CDF + lower_bound on host, in-chunk search on
// device (one wavefront per shot).  Same result as the reference's lower_bound over the full
// partial_sum except where a uniform falls within rounding distance of a CDF step.
constexpr int kChunkLog = 12;

__global__ __launch_bounds__(256) void k_chunk_sums(const double2* st, uint64_t chunk,
                                                    double* sums) {
    __shared__ double wsum[4];
    const uint64_t base = (uint64_t)blockIdx.x * chunk;
    double acc = 0.0;
    for (uint64_t i = threadIdx.x; i < chunk; i += 256) {
        const double2 a = st[base + i];
        acc += a.x * a.x + a.y * a.y;
    }
    acc = wave_sum(acc);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) sums[blockIdx.x] = (wsum[0] + wsum[1]) + (wsum[2] + wsum[3]);
}

// shot s: search chunk `chunk_of[s]` (global over the batch) for the first i with prefix >=
// target[s], output the index within its trajectory; -1 chunk -> N (the reference's end()).
__global__ __launch_bounds__(64) void k_chunk_search(const double2* st, uint64_t chunk,
                                                     const int64_t* chunk_of,
                                                     const double* target, int shots,
                                                     uint64_t total, int64_t* out) {
    const int s = blockIdx.x;
    if (s >= shots) return;
    const int64_t c = chunk_of[s];
    const int lane = threadIdx.x;
    if (c < 0) {
        if (lane == 0) out[s] = (int64_t)total;
        return;
    }
    const uint64_t base = (uint64_t)c * chunk;
    const uint64_t per = (chunk + 63) / 64;  // consecutive amplitudes per lane
    double mine = 0.0;
    for (uint64_t k = 0; k < per; ++k) {
        const uint64_t i = (uint64_t)lane * per + k;
        if (i < chunk) {
            const double2 a = st[base + i];
            mine += a.x * a.x + a.y * a.y;
        }
    }
    // inclusive wave scan of lane sums
    double incl = mine;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const double y = __shfl_up(incl, off);
        if (lane >= off) incl += y;
    }
    const double r = target[s];
    const unsigned long long ball = __ballot(incl >= r);
    int first = ball ? __ffsll((long long)ball) - 1 : 63;  // rounding: clamp to last lane
    if (lane == first) {
        double acc = incl - mine;
        uint64_t found = (uint64_t)lane * per + per - 1;
        for (uint64_t k = 0; k < per; ++k) {
            const uint64_t i = (uint64_t)lane * per + k;
            if (i >= chunk) break;
            const double2 a = st[base + i];
            acc += a.x * a.x + a.y * a.y;
            if (acc >= r) {
                found = i;
                break;
            }
        }
        if (found >= chunk) found = chunk - 1;
        out[s] = (int64_t)((base + found) & (total - 1));
    }
}

// Shots of `batch` trajectories (the single state is batch = 1).  uniforms / out are
// trajectory-major: shot s of trajectory t at t * shots + s (the reference draws them in that
// order, src/NoiseModel.cu:938-957).  The chunk prefix is accumulated with Neumaier's
// compensation, so the device CDF is the exactly rounded one up to a few ulps; an index can
// then differ from the reference's sequential partial_sum only where the uniform lies between
// the exact and the sequentially rounded CDF at a step (tests/test_sampling_gpu.py checks that).
void sample_indices(const double2* st, int n, uint64_t batch, const double* uniforms, int shots,
                    int64_t* out, hipStream_t s, Scratch& scratch) {
    if (shots <= 0 || batch == 0) return;
    const uint64_t total = 1ull << n;
    const uint64_t chunk = 1ull << std::min(n, kChunkLog);
    const uint64_t nchunks = total / chunk;  // per trajectory
    const uint64_t all_chunks = nchunks * batch;
    const uint64_t nshots = (uint64_t)shots * batch;
    // scratch = [chunk sums][chunk of shot][target of shot][index of shot], 8 B each
    char* base = (char*)scratch.get((all_chunks + 3 * nshots) * 8, s);
    double* d_sums = (double*)base;
    int64_t* d_chunk = (int64_t*)(base + all_chunks * 8);
    double* d_target = (double*)(base + (all_chunks + nshots) * 8);
    int64_t* d_out = (int64_t*)(base + (all_chunks + 2 * nshots) * 8);
    hipLaunchKernelGGL(k_chunk_sums, dim3((unsigned)all_chunks), dim3(256), 0, s, st, chunk, d_sums);
    QSIM_HIPCHK(hipGetLastError());
    std::vector<double> sums(all_chunks);
    QSIM_HIPCHK(hipMemcpyAsync(sums.data(), d_sums, all_chunks * sizeof(double),
                               hipMemcpyDeviceToHost, s));
    QSIM_HIPCHK(hipStreamSynchronize(s));
    std::vector<double> cdf(nchunks), comp(nchunks);
    std::vector<int64_t> chunk_of(nshots);
    std::vector<double> target(nshots);
    for (uint64_t t = 0; t < batch; ++t) {
        double run = 0.0, c = 0.0;  // Neumaier: run + c is the prefix to ~1 ulp
        for (uint64_t k = 0; k < nchunks; ++k) {
            const double x = sums[t * nchunks + k];
            const double y = run + x;
            c += std::fabs(run) >= std::fabs(x) ? (run - y) + x : (x - y) + run;
            run = y;
            cdf[k] = run + c;
            comp[k] = c - (cdf[k] - run);  // residual below cdf[k]
        }
        for (int i = 0; i < shots; ++i) {
            const uint64_t j = t * (uint64_t)shots + (uint64_t)i;
            const double r = uniforms[j];
            auto it = std::lower_bound(cdf.begin(), cdf.end(), r);
            if (it == cdf.end()) {
                chunk_of[j] = -1;
                target[j] = 0.0;
            } else {
                const int64_t k = it - cdf.begin();
                chunk_of[j] = (int64_t)(t * nchunks) + k;
                target[j] = k > 0 ? (r - cdf[k - 1]) - comp[k - 1] : r;
            }
        }
    }
    QSIM_HIPCHK(hipMemcpyAsync(d_chunk, chunk_of.data(), nshots * sizeof(int64_t),
                               hipMemcpyHostToDevice, s));
    QSIM_HIPCHK(hipMemcpyAsync(d_target, target.data(), nshots * sizeof(double),
                               hipMemcpyHostToDevice, s));
    for (uint64_t first = 0; first < nshots; first += 0x7fffffffull) {  // grid.x limit
        const uint64_t cnt = std::min<uint64_t>(nshots - first, 0x7fffffffull);
        hipLaunchKernelGGL(k_chunk_search, dim3((unsigned)cnt), dim3(64), 0, s, st, chunk,
                           d_chunk + first, d_target + first, (int)cnt, total, d_out + first);
        QSIM_HIPCHK(hipGetLastError());
    }
    QSIM_HIPCHK(hipMemcpyAsync(out, d_out, nshots * sizeof(int64_t), hipMemcpyDeviceToHost, s));
    QSIM_HIPCHK(hipStreamSynchronize(s));
}

// Histogram of sampled outcomes; indices >= N (the reference's end()) are skipped, as in
// BatchedSimulator::getHistogram (src/NoiseModel.cu:959-972).
__global__ __launch_bounds__(256) void k_histogram(const int64_t* idx, uint64_t count, uint64_t N,
                                                   unsigned long long* hist) {
    const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += step) {
        const int64_t o = idx[i];
        if (o >= 0 && (uint64_t)o < N) atomicAdd(hist + o, 1ull);
    }
}

void launch_histogram(const int64_t* d_idx, uint64_t count, uint64_t N, unsigned long long* d_hist,
                      hipStream_t s) {
    const uint64_t blocks = std::min<uint64_t>((count + 255) / 256, 256 * 32);
    hipLaunchKernelGGL(k_histogram, dim3((unsigned)blocks), dim3(256), 0, s, d_idx, count, N, d_hist);
    QSIM_HIPCHK(hipGetLastError());
}

// out[i] = sum_b |a_{b,i}|^2 / B, accumulated in trajectory order like the reference loop.
__global__ __launch_bounds__(256) void k_avg_probs(const double2* st, uint64_t stride,
                                                   uint64_t batch, double* out) {
    const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
    const double inv = (double)batch;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < stride; i += step) {
        double acc = 0.0;
        for (uint64_t b = 0; b < batch; ++b) {
            const double2 a = st[b * stride + i];
            acc += (a.x * a.x + a.y * a.y) / inv;
        }
        out[i] = acc;
    }
}

void launch_avg_probabilities(const double2* st, int n, uint64_t batch, double* out,
                              hipStream_t s) {
    const uint64_t stride = 1ull << n;
    const uint64_t blocks = std::min<uint64_t>((stride + 255) / 256, 256 * 32);
    hipLaunchKernelGGL(k_avg_probs, dim3((unsigned)blocks), dim3(256), 0, s, st, stride, batch,
                       out);
    QSIM_HIPCHK(hipGetLastError());
}

}  // namespace qsim_hip
