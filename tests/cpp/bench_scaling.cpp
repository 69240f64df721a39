// bench_scaling.cpp — benchmarks/benchmark_scaling.cu:58-100 (benchmarkGPUvsCPU) restated on the
// drop-in API: the W-REF circuit (h(i % n), cnot(i % n, (i+1) % n) every 5th i; 120 gates) at
// n = 10, 12, ..., 22 through qsim::Simulator (MI355X) and qsim::CPUSimulator (host), printed
// as one JSON object per n.  Differences from the reference's loop, all toward an honest
// number: the GPU time is synchronised (the reference timed asynchronous launches),
// each side is the median of `reps` runs after one warm-up, and the CPU column is reported for
// 1 thread (the reference's CPU path) and for all host threads.
#include <qsim/Circuit.hpp>
#include <qsim/Simulator.hpp>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

static double median(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? std::atoi(argv[1]) : 3;
    const int nmax = argc > 2 ? std::atoi(argv[2]) : 22;
    using clk = std::chrono::steady_clock;
    const int hw = (int)std::thread::hardware_concurrency();
    for (int n = 10; n <= nmax; n += 2) {
        const qsim::Circuit c = qsim::createScalingBenchmarkCircuit(n);
        qsim::Simulator gpu(n);
        gpu.run(c);
        gpu.synchronize();
        std::vector<double> g;
        for (int r = 0; r < reps; ++r) {
            gpu.reset();
            gpu.synchronize();
            const auto t0 = clk::now();
            gpu.run(c);
            gpu.synchronize();
            g.push_back(std::chrono::duration<double, std::milli>(clk::now() - t0).count());
        }
        double cpu_ms[2];
        const int threads[2] = {1, std::min(hw, 64)};
        for (int k = 0; k < 2; ++k) {
            qsim::CPUSimulator cpu(n);
            cpu.setThreads(threads[k]);
            cpu.run(c);
            std::vector<double> t;
            for (int r = 0; r < reps; ++r) {
                cpu.reset();
                const auto t0 = clk::now();
                cpu.run(c);
                t.push_back(std::chrono::duration<double, std::milli>(clk::now() - t0).count());
            }
            cpu_ms[k] = median(t);
        }
        std::printf("{\"qubits\": %d, \"gates\": %zu, \"gpu_ms\": %.4f, \"cpu_ms_1thread\": %.3f, "
                    "\"cpu_ms_%dthreads\": %.3f, \"speedup_vs_1thread\": %.1f}\n",
                    n, c.getGateCount(), median(g), cpu_ms[0], threads[1], cpu_ms[1],
                    cpu_ms[0] / median(g));
        std::fflush(stdout);
    }
    return 0;
}
