// Minimal syntax stub of Google Benchmark for tests/test_reference_sources.py:
// enough of the API (State, Fixture, the registration macros and their builder
// chain, Counter, DoNotOptimize, ConsoleReporter) for `g++ -fsyntax-only` to
// type-check the reference's bench/*_benchmark.cc against the drop-in headers
// (include/ref).  It stubs the harness framework, not the reference: nothing
// here runs, and no reference source is copied.
#pragma once

#include <cstdint>
#include <map>
#include <string>
#include <vector>

namespace benchmark {

enum TimeUnit { kNanosecond, kMicrosecond, kMillisecond, kSecond };

struct Counter {
    enum Flags { kDefaults = 0, kIsRate = 1, kAvgThreads = 2, kAvgIterations = 4, kIsIterationInvariantRate = 8 };
    double value = 0;
    Counter(double v = 0.0, Flags = kDefaults) : value(v) {}
    operator double() const { return value; }
};

class State {
public:
    struct Iter {
        int64_t left = 0;
        bool operator!=(const Iter& o) const { return left != o.left; }
        Iter& operator++() { --left; return *this; }
        int operator*() const { return 0; }
    };
    Iter begin() { return Iter{0}; }
    Iter end() { return Iter{0}; }
    bool KeepRunning() { return false; }
    int64_t range(std::size_t = 0) const { return 0; }
    int64_t iterations() const { return 0; }
    int64_t max_iterations = 0;
    int threads() const { return 1; }
    int thread_index() const { return 0; }
    void SetItemsProcessed(int64_t) {}
    void SetBytesProcessed(int64_t) {}
    void SetIterationTime(double) {}
    void SetLabel(const std::string&) {}
    void SkipWithError(const std::string&) {}
    void PauseTiming() {}
    void ResumeTiming() {}
    std::map<std::string, Counter> counters;
};

template <class T>
inline void DoNotOptimize(T&&) {}
inline void ClobberMemory() {}

namespace internal {
class Benchmark {
public:
    virtual ~Benchmark() = default;
    Benchmark* Arg(int64_t) { return this; }
    Benchmark* Args(const std::vector<int64_t>&) { return this; }
    Benchmark* ArgsProduct(const std::vector<std::vector<int64_t>>&) { return this; }
    Benchmark* ArgName(const std::string&) { return this; }
    Benchmark* ArgNames(const std::vector<std::string>&) { return this; }
    Benchmark* Range(int64_t, int64_t) { return this; }
    Benchmark* RangeMultiplier(int) { return this; }
    Benchmark* DenseRange(int64_t, int64_t, int = 1) { return this; }
    Benchmark* Ranges(const std::vector<std::pair<int64_t, int64_t>>&) { return this; }
    Benchmark* Unit(TimeUnit) { return this; }
    Benchmark* Iterations(int64_t) { return this; }
    Benchmark* Repetitions(int) { return this; }
    Benchmark* MinTime(double) { return this; }
    Benchmark* UseRealTime() { return this; }
    Benchmark* UseManualTime() { return this; }
    Benchmark* Threads(int) { return this; }
    Benchmark* ThreadRange(int, int) { return this; }
    Benchmark* Name(const std::string&) { return this; }
    Benchmark* Apply(void (*)(Benchmark*)) { return this; }
};
inline Benchmark* RegisterFn(const char*, void (*)(State&)) {
    static Benchmark b;
    return &b;
}
}  // namespace internal

class Fixture : public internal::Benchmark {
public:
    virtual void SetUp(const State&) {}
    virtual void TearDown(const State&) {}
    virtual void SetUp(State& st) { SetUp(static_cast<const State&>(st)); }
    virtual void TearDown(State& st) { TearDown(static_cast<const State&>(st)); }
    virtual void BenchmarkCase(State&) {}
};

struct BenchmarkReporter {
    struct Context {};
    struct Run {
        std::string benchmark_name() const { return {}; }
        double GetAdjustedRealTime() const { return 0; }
        double GetAdjustedCPUTime() const { return 0; }
        int64_t iterations = 0;
        TimeUnit time_unit = kNanosecond;
        std::map<std::string, Counter> counters;
        std::string report_label;
        bool error_occurred = false;
    };
    virtual ~BenchmarkReporter() = default;
    virtual bool ReportContext(const Context&) { return true; }
    virtual void ReportRuns(const std::vector<Run>&) {}
    virtual void Finalize() {}
};
class ConsoleReporter : public BenchmarkReporter {
public:
    bool ReportContext(const Context&) override { return true; }
    void ReportRuns(const std::vector<Run>&) override {}
};

inline void Initialize(int*, char**) {}
inline bool ReportUnrecognizedArguments(int, char**) { return false; }
inline std::size_t RunSpecifiedBenchmarks() { return 0; }
inline std::size_t RunSpecifiedBenchmarks(BenchmarkReporter*) { return 0; }
inline void Shutdown() {}

}  // namespace benchmark

#define CRLOT_BM_CAT2(a, b) a##b
#define CRLOT_BM_CAT(a, b) CRLOT_BM_CAT2(a, b)
#define BENCHMARK(fn) \
    static ::benchmark::internal::Benchmark* CRLOT_BM_CAT(crlot_bm_, __LINE__) = ::benchmark::internal::RegisterFn(#fn, fn)
#define BENCHMARK_DEFINE_F(fixture, name)                               \
    struct fixture##_##name##_Benchmark : fixture {                     \
        void BenchmarkCase(::benchmark::State&) override;               \
    };                                                                  \
    void fixture##_##name##_Benchmark::BenchmarkCase
#define BENCHMARK_REGISTER_F(fixture, name) \
    static ::benchmark::internal::Benchmark* CRLOT_BM_CAT(crlot_bmf_, __LINE__) = (new fixture##_##name##_Benchmark())
#define BENCHMARK_F(fixture, name)                                      \
    BENCHMARK_DEFINE_F(fixture, name)(::benchmark::State&);             \
    BENCHMARK_REGISTER_F(fixture, name);                                \
    void fixture##_##name##_Benchmark::BenchmarkCase
#define BENCHMARK_MAIN()                          \
    int main(int argc, char** argv) {             \
        ::benchmark::Initialize(&argc, argv);     \
        ::benchmark::RunSpecifiedBenchmarks();    \
        return 0;                                 \
    }
