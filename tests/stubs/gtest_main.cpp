// main() and the runner of the gtest work-alike (tests/stubs/gtest/gtest.h):
// runs every registered test (or those whose "Suite.Name" contains argv[1]),
// prints one line per test and a JSON summary line last; exit status 1 when any
// test failed.
#include <cstring>
#include <exception>

#include "gtest/gtest.h"

int RUN_ALL_TESTS_impl() { return 0; }

int main(int argc, char** argv) {
    using namespace testing::internal;
    const char* filter = argc > 1 ? argv[1] : nullptr;
    int run = 0, failed = 0;
    std::string failed_names;
    for (auto& t : registry()) {
        const std::string full = t.suite + "." + t.name;
        if (filter && !std::strstr(full.c_str(), filter)) continue;
        current_test() = full;
        failures_in_test() = 0;
        ++run;
        try {
            std::unique_ptr<testing::Test> obj(t.make());
            obj->SetUp();
            if (failures_in_test() == 0) obj->TestBody();
            obj->TearDown();
        } catch (const std::exception& e) {
            ++failures_in_test();
            std::printf("%s: uncaught exception: %s\n", full.c_str(), e.what());
        } catch (...) {
            ++failures_in_test();
            std::printf("%s: uncaught exception\n", full.c_str());
        }
        const bool ok = failures_in_test() == 0;
        std::printf("[%s] %s\n", ok ? "  OK  " : "FAILED", full.c_str());
        std::fflush(stdout);
        if (!ok) {
            ++failed;
            failed_names += (failed_names.empty() ? "\"" : ", \"") + full + "\"";
        }
    }
    std::printf("{\"tests\": %d, \"failed\": %d, \"failed_names\": [%s]}\n", run, failed, failed_names.c_str());
    return failed ? 1 : 0;
}
