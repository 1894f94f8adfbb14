// Minimal syntax stub of GoogleTest for tests/test_reference_sources.py: enough of
// the API (TEST / TEST_F, ::testing::Test, the EXPECT_ / ASSERT_ macros) for
// `g++ -fsyntax-only` to type-check the reference's gtest files against the
// drop-in headers (include/ref).  It stubs the test framework, not the
// reference: nothing here runs, and no reference source is copied.
#pragma once

// (the headers real gtest.h brings in transitively, which test files rely on)
#include <cmath>
#include <iostream>
#include <map>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

namespace testing {

class Test {
public:
    virtual ~Test() = default;
    virtual void TestBody() {}

protected:
    virtual void SetUp() {}
    virtual void TearDown() {}
};

// the object an assertion macro yields, so that `EXPECT_EQ(a, b) << "note"` parses
struct Message {
    template <class T>
    Message& operator<<(const T&) { return *this; }
};
template <class... T>
inline Message check(const T&...) { return Message{}; }
template <class A, class B>
inline bool eq(const A& a, const B& b) { return a == b; }
template <class A, class B>
inline bool ne(const A& a, const B& b) { return a != b; }
template <class A, class B>
inline bool lt(const A& a, const B& b) { return a < b; }
template <class A, class B>
inline bool le(const A& a, const B& b) { return a <= b; }
template <class A, class B>
inline bool gt(const A& a, const B& b) { return a > b; }
template <class A, class B>
inline bool ge(const A& a, const B& b) { return a >= b; }
template <class A, class B, class C>
inline bool near(const A& a, const B& b, const C& tol) { return std::fabs(double(a) - double(b)) <= double(tol); }

inline void InitGoogleTest(int*, char**) {}

}  // namespace testing

#define CRLOT_STUB_CAT2(a, b) a##b
#define CRLOT_STUB_CAT(a, b) CRLOT_STUB_CAT2(a, b)

#define TEST(suite, name)                                            \
    struct suite##_##name##_Test : ::testing::Test {                 \
        void TestBody() override;                                    \
    };                                                               \
    void suite##_##name##_Test::TestBody()
#define TEST_F(fixture, name)                                        \
    struct fixture##_##name##_Test : fixture {                       \
        void TestBody() override;                                    \
    };                                                               \
    void fixture##_##name##_Test::TestBody()

#define EXPECT_TRUE(c) ::testing::check(bool(c))
#define EXPECT_FALSE(c) ::testing::check(!(c))
#define EXPECT_EQ(a, b) ::testing::check(::testing::eq((a), (b)))
#define EXPECT_NE(a, b) ::testing::check(::testing::ne((a), (b)))
#define EXPECT_LT(a, b) ::testing::check(::testing::lt((a), (b)))
#define EXPECT_LE(a, b) ::testing::check(::testing::le((a), (b)))
#define EXPECT_GT(a, b) ::testing::check(::testing::gt((a), (b)))
#define EXPECT_GE(a, b) ::testing::check(::testing::ge((a), (b)))
#define EXPECT_NEAR(a, b, t) ::testing::check(::testing::near((a), (b), (t)))
#define EXPECT_FLOAT_EQ(a, b) ::testing::check(::testing::eq(float(a), float(b)))
#define EXPECT_DOUBLE_EQ(a, b) ::testing::check(::testing::eq(double(a), double(b)))
#define EXPECT_STREQ(a, b) ::testing::check(std::string(a) == std::string(b))
#define EXPECT_THROW(stmt, exc) ::testing::check([&]() { try { stmt; } catch (const exc&) {} })
#define EXPECT_NO_THROW(stmt) ::testing::check([&]() { stmt; })
#define EXPECT_ANY_THROW(stmt) ::testing::check([&]() { try { stmt; } catch (...) {} })
#define ASSERT_TRUE EXPECT_TRUE
#define ASSERT_FALSE EXPECT_FALSE
#define ASSERT_EQ EXPECT_EQ
#define ASSERT_NE EXPECT_NE
#define ASSERT_LT EXPECT_LT
#define ASSERT_LE EXPECT_LE
#define ASSERT_GT EXPECT_GT
#define ASSERT_GE EXPECT_GE
#define ASSERT_NEAR EXPECT_NEAR
#define ASSERT_FLOAT_EQ EXPECT_FLOAT_EQ
#define ASSERT_THROW EXPECT_THROW
#define ASSERT_NO_THROW EXPECT_NO_THROW
#define GTEST_SKIP() return (void)::testing::Message()
#define SCOPED_TRACE(m) (void)(m)
#define RUN_ALL_TESTS() 0
