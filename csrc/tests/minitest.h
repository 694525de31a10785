// Minimal gtest-style unit test harness (gtest is not available in this image).
// TEST(Suite, Name) registers a case; EXPECT_* record failures; ASSERT_* abort the case.
// The runner supports --filter=<substring> and prints one line per case.
#pragma once

#include <cmath>
#include <cstdio>
#include <cstring>
#include <functional>
#include <sstream>
#include <string>
#include <type_traits>
#include <vector>

namespace minitest {

struct Case {
  std::string name;
  std::function<void()> fn;
};
inline std::vector<Case>& Registry() {
  static std::vector<Case> r;
  return r;
}
inline int& Failures() {
  static int f = 0;
  return f;
}
struct AssertAbort {};
struct Registrar {
  Registrar(const char* suite, const char* name, std::function<void()> fn) {
    Registry().push_back({std::string(suite) + "." + name, std::move(fn)});
  }
};
inline void Fail(const char* file, int line, const std::string& msg) {
  std::fprintf(stderr, "  %s:%d: %s\n", file, line, msg.c_str());
  Failures()++;
}

template <typename T, typename = void>
struct IsStreamable : std::false_type {};
template <typename T>
struct IsStreamable<T, std::void_t<decltype(std::declval<std::ostream&>() << std::declval<const T&>())>>
    : std::true_type {};

template <typename T>
std::string Show(const T& v) {
  std::ostringstream os;
  if constexpr (std::is_enum<T>::value) {
    os << static_cast<long long>(v);
  } else if constexpr (std::is_arithmetic<T>::value) {
    os << +v;
  } else if constexpr (IsStreamable<T>::value) {
    os << v;
  } else {
    os << "<value>";
  }
  return os.str();
}

inline int RunAll(int argc, char** argv) {
  std::string filter;
  for (int i = 1; i < argc; ++i)
    if (std::strncmp(argv[i], "--filter=", 9) == 0) filter = argv[i] + 9;
  int failed_cases = 0, ran = 0;
  for (auto& c : Registry()) {
    if (!filter.empty() && c.name.find(filter) == std::string::npos) continue;
    int before = Failures();
    try {
      c.fn();
    } catch (const AssertAbort&) {
    } catch (const std::exception& e) {
      Fail(__FILE__, __LINE__, std::string("uncaught exception: ") + e.what());
    }
    ++ran;
    bool ok = Failures() == before;
    if (!ok) ++failed_cases;
    std::printf("[%s] %s\n", ok ? "  OK  " : " FAIL ", c.name.c_str());
    std::fflush(stdout);
  }
  std::printf("%d/%d cases passed\n", ran - failed_cases, ran);
  return failed_cases == 0 && ran > 0 ? 0 : 1;
}

}  // namespace minitest

#define MT_CAT2(a, b) a##b
#define MT_CAT(a, b) MT_CAT2(a, b)
#define TEST(suite, name)                                                                    \
  static void suite##_##name##_impl();                                                       \
  static ::minitest::Registrar MT_CAT(reg_##suite##_##name, __LINE__)(#suite, #name,         \
                                                                      suite##_##name##_impl); \
  static void suite##_##name##_impl()

#define MT_CHECK_OP(a, b, op, fatal)                                                   \
  do {                                                                                 \
    const auto _a = (a);                                                                \
    const auto _b = (b);                                                                \
    if (!(_a op _b)) {                                                                 \
      std::ostringstream _os;                                                          \
      _os << #a " " #op " " #b " failed: " << ::minitest::Show(_a) << " vs " << ::minitest::Show(_b);                  \
      ::minitest::Fail(__FILE__, __LINE__, _os.str());                                 \
      if (fatal) throw ::minitest::AssertAbort();                                      \
    }                                                                                  \
  } while (0)

#define EXPECT_EQ(a, b) MT_CHECK_OP(a, b, ==, false)
#define EXPECT_NE(a, b) MT_CHECK_OP(a, b, !=, false)
#define EXPECT_LT(a, b) MT_CHECK_OP(a, b, <, false)
#define EXPECT_LE(a, b) MT_CHECK_OP(a, b, <=, false)
#define EXPECT_GT(a, b) MT_CHECK_OP(a, b, >, false)
#define EXPECT_GE(a, b) MT_CHECK_OP(a, b, >=, false)
#define ASSERT_EQ(a, b) MT_CHECK_OP(a, b, ==, true)
#define ASSERT_NE(a, b) MT_CHECK_OP(a, b, !=, true)
#define ASSERT_GE(a, b) MT_CHECK_OP(a, b, >=, true)
#define EXPECT_TRUE(a) MT_CHECK_OP((bool)(a), true, ==, false)
#define EXPECT_FALSE(a) MT_CHECK_OP((bool)(a), false, ==, false)
#define ASSERT_TRUE(a) MT_CHECK_OP((bool)(a), true, ==, true)
#define EXPECT_DOUBLE_EQ(a, b) \
  MT_CHECK_OP(std::fabs((double)(a) - (double)(b)) <= 1e-12 * (1 + std::fabs((double)(b))), true, ==, false)
#define EXPECT_NEAR(a, b, tol) MT_CHECK_OP(std::fabs((double)(a) - (double)(b)) <= (tol), true, ==, false)
#define EXPECT_THROW(stmt)                                                     \
  do {                                                                         \
    bool _thrown = false;                                                      \
    try {                                                                      \
      stmt;                                                                    \
    } catch (...) {                                                            \
      _thrown = true;                                                          \
    }                                                                          \
    if (!_thrown) ::minitest::Fail(__FILE__, __LINE__, #stmt " did not throw"); \
  } while (0)
