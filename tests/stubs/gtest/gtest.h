// A small GoogleTest work-alike for running the reference's own gtest files
// against the drop-in (tests/reftests/Makefile, tests/test_reference_sources.py,
// tests/test_gpu_reference_suites.py): TEST / TEST_F with
// ::testing::Test fixtures (SetUp / TearDown), the EXPECT_ / ASSERT_ families
// with streamed messages, EXPECT_THROW / NO_THROW, and RUN_ALL_TESTS.  A
// failed EXPECT records and continues, a failed ASSERT records and returns
// from the test body, an escaping exception fails the test.  Link with
// gtest_main.cpp (as the reference links gtest_main).  This re-implements the
// test framework's API, not any reference code.
#pragma once

// (the headers real gtest.h brings in transitively, which test files rely on)
#include <cmath>
#include <cstdio>
#include <functional>
#include <iostream>
#include <map>
#include <memory>
#include <sstream>
#include <string>
#include <utility>
#include <vector>

namespace testing {

class Test {
public:
    virtual ~Test() = default;
    virtual void TestBody() = 0;
    virtual void SetUp() {}
    virtual void TearDown() {}
};

class Message {
public:
    Message() = default;
    Message(const Message& o) : ss_(o.ss_.str()) {}
    template <class T>
    Message& operator<<(const T& v) {
        ss_ << v;
        return *this;
    }
    std::string str() const { return ss_.str(); }

private:
    std::ostringstream ss_;
};

namespace internal {

struct TestInfo {
    std::string suite, name;
    std::function<Test*()> make;
};
inline std::vector<TestInfo>& registry() {
    static std::vector<TestInfo> r;
    return r;
}
struct Registrar {
    Registrar(const char* s, const char* n, std::function<Test*()> f) { registry().push_back({s, n, std::move(f)}); }
};
inline int& failures_in_test() {
    static int n = 0;
    return n;
}
inline std::string& current_test() {
    static std::string s;
    return s;
}

// `AssertHelper(...) = Message() << ...` records one failure; the assignment
// returns void so `return AssertHelper(...) = Message()` leaves a void function.
class AssertHelper {
public:
    AssertHelper(const char* file, int line, std::string what) : file_(file), line_(line), what_(std::move(what)) {}
    void operator=(const Message& m) const {
        ++failures_in_test();
        std::fprintf(stdout, "%s:%d: Failure in %s\n  %s%s%s\n", file_, line_, current_test().c_str(), what_.c_str(),
                     m.str().empty() ? "" : "\n  ", m.str().c_str());
        std::fflush(stdout);
    }

private:
    const char* file_;
    int line_;
    std::string what_;
};

template <class T>
auto print_one(std::ostream& os, const T& v, int) -> decltype(os << v, void()) {
    os << v;
}
template <class T>
void print_one(std::ostream& os, const T&, long) {
    os << "<value>";
}
template <class T>
std::string show(const T& v) {
    std::ostringstream os;
    print_one(os, v, 0);
    return os.str();
}
template <class A, class B>
std::string cmp_text(const char* ea, const char* eb, const char* op, const A& a, const B& b) {
    return std::string("Expected: (") + ea + ") " + op + " (" + eb + "), actual: " + show(a) + " vs " + show(b);
}

// plain comparisons (a signed / unsigned mix compares as the values say, not as the promotions)
template <class A, class B>
bool eq(const A& a, const B& b) {
    if constexpr (std::is_integral<A>::value && std::is_integral<B>::value && std::is_signed<A>::value !=
                  std::is_signed<B>::value) {
        using W = long double;
        return W(a) == W(b);
    } else {
        return a == b;
    }
}
inline bool float_eq(double a, double b, bool single) {
    // within 4 ULPs (gtest's FloatingPointEq)
    if (std::isnan(a) || std::isnan(b)) return false;
    if (a == b) return true;
    const double ulp = single ? std::fabs(double(std::nextafter(float(a), float(b))) - a)
                              : std::fabs(std::nextafter(a, b) - a);
    return std::fabs(a - b) <= 4 * ulp;
}

}  // namespace internal

inline void InitGoogleTest(int*, char**) {}
inline void InitGoogleTest() {}

}  // namespace testing

int RUN_ALL_TESTS_impl();
#define RUN_ALL_TESTS() RUN_ALL_TESTS_impl()

#define CRLOT_GT_CAT2(a, b) a##b
#define CRLOT_GT_CAT(a, b) CRLOT_GT_CAT2(a, b)

#define CRLOT_GT_TEST_(suite, name, base)                                                              \
    struct suite##_##name##_Test : base {                                                              \
        void TestBody() override;                                                                      \
    };                                                                                                 \
    static ::testing::internal::Registrar CRLOT_GT_CAT(crlot_gt_reg_, __LINE__)(                       \
        #suite, #name, [] { return static_cast<::testing::Test*>(new suite##_##name##_Test()); });     \
    void suite##_##name##_Test::TestBody()
#define TEST(suite, name) CRLOT_GT_TEST_(suite, name, ::testing::Test)
#define TEST_F(fixture, name) CRLOT_GT_TEST_(fixture, name, fixture)

#define CRLOT_GT_FAIL_(what, fatal) \
    fatal ::testing::internal::AssertHelper(__FILE__, __LINE__, what) = ::testing::Message()
#define CRLOT_GT_CHECK_(cond, what, fatal) \
    switch (0)                             \
    case 0:                                \
    default:                               \
        if (cond)                          \
            ;                              \
        else                               \
            CRLOT_GT_FAIL_(what, fatal)
#define CRLOT_GT_BOOL_(c, expect, fatal) \
    CRLOT_GT_CHECK_(bool(c) == expect, std::string("Value of: ") + #c + (expect ? " is false" : " is true"), fatal)
#define CRLOT_GT_CMP_(a, b, op, fatal)                                                                            \
    CRLOT_GT_CHECK_(([&] {                                                                                        \
                        const auto& crlot_a_ = (a);                                                               \
                        const auto& crlot_b_ = (b);                                                               \
                        return op;                                                                                \
                    }()),                                                                                          \
                    ::testing::internal::cmp_text(#a, #b, #op, (a), (b)), fatal)
#define CRLOT_GT_NEAR_(a, b, t, fatal)                                                                          \
    CRLOT_GT_CHECK_(std::fabs(double(a) - double(b)) <= double(t),                                              \
                    ::testing::internal::cmp_text(#a, #b, "near", double(a), double(b)) + " tol " + std::to_string(double(t)), fatal)
#define CRLOT_GT_FEQ_(a, b, single, fatal) \
    CRLOT_GT_CHECK_(::testing::internal::float_eq(double(a), double(b), single), \
                    ::testing::internal::cmp_text(#a, #b, "float-eq", double(a), double(b)), fatal)
#define CRLOT_GT_THROW_(stmt, exc, fatal)                                              \
    CRLOT_GT_CHECK_(([&] {                                                             \
                        try {                                                          \
                            stmt;                                                      \
                        } catch (const exc&) {                                         \
                            return true;                                               \
                        } catch (...) {                                                \
                            return false;                                              \
                        }                                                              \
                        return false;                                                  \
                    }()),                                                              \
                    std::string("Expected: ") + #stmt + " throws " + #exc, fatal)
#define CRLOT_GT_NOTHROW_(stmt, fatal)                                                 \
    CRLOT_GT_CHECK_(([&] {                                                             \
                        try {                                                          \
                            stmt;                                                      \
                        } catch (...) {                                                \
                            return false;                                              \
                        }                                                              \
                        return true;                                                   \
                    }()),                                                              \
                    std::string("Expected: ") + #stmt + " does not throw", fatal)
#define CRLOT_GT_ANYTHROW_(stmt, fatal)                                                \
    CRLOT_GT_CHECK_(([&] {                                                             \
                        try {                                                          \
                            stmt;                                                      \
                        } catch (...) {                                                \
                            return true;                                               \
                        }                                                              \
                        return false;                                                  \
                    }()),                                                              \
                    std::string("Expected: ") + #stmt + " throws", fatal)

#define CRLOT_GT_NF_
#define CRLOT_GT_F_ return

#define EXPECT_TRUE(c) CRLOT_GT_BOOL_(c, true, CRLOT_GT_NF_)
#define EXPECT_FALSE(c) CRLOT_GT_BOOL_(c, false, CRLOT_GT_NF_)
#define EXPECT_EQ(a, b) CRLOT_GT_CMP_(a, b, ::testing::internal::eq(crlot_a_, crlot_b_), CRLOT_GT_NF_)
#define EXPECT_NE(a, b) CRLOT_GT_CMP_(a, b, !::testing::internal::eq(crlot_a_, crlot_b_), CRLOT_GT_NF_)
#define EXPECT_LT(a, b) CRLOT_GT_CMP_(a, b, crlot_a_ < crlot_b_, CRLOT_GT_NF_)
#define EXPECT_LE(a, b) CRLOT_GT_CMP_(a, b, crlot_a_ <= crlot_b_, CRLOT_GT_NF_)
#define EXPECT_GT(a, b) CRLOT_GT_CMP_(a, b, crlot_a_ > crlot_b_, CRLOT_GT_NF_)
#define EXPECT_GE(a, b) CRLOT_GT_CMP_(a, b, crlot_a_ >= crlot_b_, CRLOT_GT_NF_)
#define EXPECT_NEAR(a, b, t) CRLOT_GT_NEAR_(a, b, t, CRLOT_GT_NF_)
#define EXPECT_FLOAT_EQ(a, b) CRLOT_GT_FEQ_(a, b, true, CRLOT_GT_NF_)
#define EXPECT_DOUBLE_EQ(a, b) CRLOT_GT_FEQ_(a, b, false, CRLOT_GT_NF_)
#define EXPECT_STREQ(a, b) CRLOT_GT_CHECK_(std::string(a) == std::string(b), std::string(#a " == " #b), CRLOT_GT_NF_)
#define EXPECT_STRNE(a, b) CRLOT_GT_CHECK_(std::string(a) != std::string(b), std::string(#a " != " #b), CRLOT_GT_NF_)
#define ASSERT_STREQ(a, b) CRLOT_GT_CHECK_(std::string(a) == std::string(b), std::string(#a " == " #b), CRLOT_GT_F_)
#define EXPECT_THROW(stmt, exc) CRLOT_GT_THROW_(stmt, exc, CRLOT_GT_NF_)
#define EXPECT_NO_THROW(stmt) CRLOT_GT_NOTHROW_(stmt, CRLOT_GT_NF_)
#define EXPECT_ANY_THROW(stmt) CRLOT_GT_ANYTHROW_(stmt, CRLOT_GT_NF_)
#define ASSERT_TRUE(c) CRLOT_GT_BOOL_(c, true, CRLOT_GT_F_)
#define ASSERT_FALSE(c) CRLOT_GT_BOOL_(c, false, CRLOT_GT_F_)
#define ASSERT_EQ(a, b) CRLOT_GT_CMP_(a, b, ::testing::internal::eq(crlot_a_, crlot_b_), CRLOT_GT_F_)
#define ASSERT_NE(a, b) CRLOT_GT_CMP_(a, b, !::testing::internal::eq(crlot_a_, crlot_b_), CRLOT_GT_F_)
#define ASSERT_LT(a, b) CRLOT_GT_CMP_(a, b, crlot_a_ < crlot_b_, CRLOT_GT_F_)
#define ASSERT_LE(a, b) CRLOT_GT_CMP_(a, b, crlot_a_ <= crlot_b_, CRLOT_GT_F_)
#define ASSERT_GT(a, b) CRLOT_GT_CMP_(a, b, crlot_a_ > crlot_b_, CRLOT_GT_F_)
#define ASSERT_GE(a, b) CRLOT_GT_CMP_(a, b, crlot_a_ >= crlot_b_, CRLOT_GT_F_)
#define ASSERT_NEAR(a, b, t) CRLOT_GT_NEAR_(a, b, t, CRLOT_GT_F_)
#define ASSERT_FLOAT_EQ(a, b) CRLOT_GT_FEQ_(a, b, true, CRLOT_GT_F_)
#define ASSERT_DOUBLE_EQ(a, b) CRLOT_GT_FEQ_(a, b, false, CRLOT_GT_F_)
#define ASSERT_THROW(stmt, exc) CRLOT_GT_THROW_(stmt, exc, CRLOT_GT_F_)
#define ASSERT_NO_THROW(stmt) CRLOT_GT_NOTHROW_(stmt, CRLOT_GT_F_)
#define ASSERT_ANY_THROW(stmt) CRLOT_GT_ANYTHROW_(stmt, CRLOT_GT_F_)
#define ADD_FAILURE() CRLOT_GT_FAIL_("ADD_FAILURE", CRLOT_GT_NF_)
#define FAIL() CRLOT_GT_FAIL_("FAIL", CRLOT_GT_F_)
#define SUCCEED() ::testing::Message()
#define GTEST_SKIP() return (void)(::testing::Message())
#define SCOPED_TRACE(m) (void)(m)
