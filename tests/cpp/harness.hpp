// harness.hpp — minimal self-contained test harness for the C++ API tests (GoogleTest cannot be
// fetched offline).  TEST(suite, name) registers a case; EXPECT_* record failures and
// continue, ASSERT_* abort the case.  main() runs every case (or those whose "suite.name"
// contains argv[1]) and returns the number of failed cases.
#pragma once

#include <cmath>
#include <complex>
#include <cstdio>
#include <cstring>
#include <exception>
#include <functional>
#include <string>
#include <vector>

namespace th {

struct Case {
    const char* suite;
    const char* name;
    std::function<void()> fn;
};
inline std::vector<Case>& registry() {
    static std::vector<Case> r;
    return r;
}
struct Reg {
    Reg(const char* s, const char* n, std::function<void()> f) { registry().push_back({s, n, std::move(f)}); }
};
struct Abort {};
inline int& failures() {
    static int f = 0;
    return f;
}
inline void fail(const char* file, int line, const std::string& msg) {
    ++failures();
    std::fprintf(stderr, "  %s:%d: %s\n", file, line, msg.c_str());
}

}  // namespace th

#define TH_CAT2(a, b) a##b
#define TH_CAT(a, b) TH_CAT2(a, b)
#define TEST(suite, name)                                                                   \
    static void TH_CAT(th_case_, TH_CAT(suite, name))();                                   \
    static th::Reg TH_CAT(th_reg_, TH_CAT(suite, name))(#suite, #name,                      \
                                                        TH_CAT(th_case_, TH_CAT(suite, name))); \
    static void TH_CAT(th_case_, TH_CAT(suite, name))()

#define EXPECT_TRUE(c) \
    do { if (!(c)) th::fail(__FILE__, __LINE__, "expected: " #c); } while (0)
#define ASSERT_TRUE(c) \
    do { if (!(c)) { th::fail(__FILE__, __LINE__, "required: " #c); throw th::Abort{}; } } while (0)
#define EXPECT_EQ(a, b)                                                                     \
    do {                                                                                    \
        if (!((a) == (b))) th::fail(__FILE__, __LINE__, "expected " #a " == " #b);           \
    } while (0)
#define EXPECT_NEAR(a, b, tol)                                                              \
    do {                                                                                    \
        const double th_a = (a), th_b = (b);                                                \
        if (!(std::fabs(th_a - th_b) <= (tol))) {                                           \
            char th_buf[256];                                                               \
            std::snprintf(th_buf, sizeof th_buf, "|%s - %s| = |%.17g - %.17g| > %g", #a, #b, \
                          th_a, th_b, (double)(tol));                                        \
            th::fail(__FILE__, __LINE__, th_buf);                                           \
        }                                                                                   \
    } while (0)
#define EXPECT_THROW(stmt, ex)                                                              \
    do {                                                                                    \
        bool th_ok = false;                                                                 \
        try { stmt; } catch (const ex&) { th_ok = true; } catch (...) {}                   \
        if (!th_ok) th::fail(__FILE__, __LINE__, "expected " #stmt " to throw " #ex);       \
    } while (0)
#define EXPECT_NO_THROW(stmt)                                                               \
    do {                                                                                    \
        try { stmt; } catch (const std::exception& e) {                                     \
            th::fail(__FILE__, __LINE__, std::string("unexpected exception: ") + e.what()); \
        }                                                                                   \
    } while (0)

#define TH_MAIN                                                                             \
    int main(int argc, char** argv) {                                                       \
        int failed_cases = 0, run = 0;                                                      \
        for (const th::Case& c : th::registry()) {                                          \
            const std::string id = std::string(c.suite) + "." + c.name;                     \
            if (argc > 1 && id.find(argv[1]) == std::string::npos) continue;                \
            const int before = th::failures();                                              \
            ++run;                                                                          \
            try { c.fn(); } catch (const th::Abort&) {                                      \
            } catch (const std::exception& e) {                                             \
                th::fail(__FILE__, __LINE__, std::string("uncaught: ") + e.what());         \
            }                                                                               \
            const bool ok = th::failures() == before;                                       \
            if (!ok) ++failed_cases;                                                        \
            std::printf("[%s] %s\n", ok ? "  OK  " : " FAIL ", id.c_str());                  \
        }                                                                                   \
        std::printf("%d cases, %d failed\n", run, failed_cases);                            \
        return failed_cases;                                                                \
    }
