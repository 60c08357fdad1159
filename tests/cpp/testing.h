/*!
 * \file tests/cpp/testing.h
 * \brief Minimal in-repo unit-test harness (gtest is not installed on the
 *  build image): TEST registration, EXPECT/ASSERT macros,
 *  fork-based death tests, `--filter=substr` and `--list` on the command line.
 */
#ifndef DMLC_TESTS_CPP_TESTING_H_
#define DMLC_TESTS_CPP_TESTING_H_

#include <sys/wait.h>
#include <unistd.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

namespace testing {

struct TestCase {
  std::string name;
  std::function<void()> body;
};

inline std::vector<TestCase>& Registry() {
  static std::vector<TestCase> tests;
  return tests;
}

struct Registrar {
  Registrar(const char* suite, const char* name, std::function<void()> body) {
    Registry().push_back({std::string(suite) + "." + name, std::move(body)});
  }
};

/*! \brief thrown by ASSERT_* to abort the current test */
struct AssertionAbort {};

inline int& Failures() {
  static int failures = 0;
  return failures;
}

inline void ReportFailure(const char* file, int line, const std::string& msg) {
  ++Failures();
  std::cerr << file << ":" << line << ": Failure\n  " << msg << std::endl;
}

/*! \brief run `fn` in a forked child; true if the child died (signal or non-zero exit) */
inline bool DiesInChild(const std::function<void()>& fn) {
  std::fflush(nullptr);
  pid_t pid = fork();
  if (pid == 0) {
    // silence the child's diagnostics
    if (std::freopen("/dev/null", "w", stderr) == nullptr) _exit(3);
    try {
      fn();
    } catch (...) {
      std::abort();
    }
    _exit(0);
  }
  int status = 0;
  waitpid(pid, &status, 0);
  return WIFSIGNALED(status) || (WIFEXITED(status) && WEXITSTATUS(status) != 0);
}

inline int RunAll(int argc, char** argv) {
  std::string filter;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a.rfind("--filter=", 0) == 0) filter = a.substr(9);
    if (a == "--list") {
      for (auto& t : Registry()) std::cout << t.name << "\n";
      return 0;
    }
  }
  int run = 0, failed = 0;
  std::vector<std::string> failed_names;
  for (auto& t : Registry()) {
    if (!filter.empty() && t.name.find(filter) == std::string::npos) continue;
    ++run;
    int before = Failures();
    std::cout << "[ RUN      ] " << t.name << std::endl;
    try {
      t.body();
    } catch (const AssertionAbort&) {
    } catch (const std::exception& e) {
      ReportFailure(__FILE__, __LINE__, std::string("uncaught exception: ") + e.what());
    }
    if (Failures() != before) {
      ++failed;
      failed_names.push_back(t.name);
      std::cout << "[  FAILED  ] " << t.name << std::endl;
    } else {
      std::cout << "[       OK ] " << t.name << std::endl;
    }
  }
  std::cout << "[==========] " << run << " tests, " << failed << " failed" << std::endl;
  for (auto& n : failed_names) std::cout << "[  FAILED  ] " << n << std::endl;
  return failed == 0 && run > 0 ? 0 : 1;
}

}  // namespace testing

#define TEST(suite, name)                                                           \
  static void suite##_##name##_body();                                              \
  static ::testing::Registrar suite##_##name##_registrar(#suite, #name,             \
                                                         suite##_##name##_body);    \
  static void suite##_##name##_body()

#define TESTING_CHECK_(cond, fatal, text)                                           \
  do {                                                                              \
    if (!(cond)) {                                                                  \
      std::ostringstream os_;                                                       \
      os_ << text;                                                                  \
      ::testing::ReportFailure(__FILE__, __LINE__, os_.str());                      \
      if (fatal) throw ::testing::AssertionAbort();                                 \
    }                                                                               \
  } while (0)

#define TESTING_CMP_(a, b, op, fatal)                                               \
  do {                                                                              \
    const auto& va_ = (a);                                                          \
    const auto& vb_ = (b);                                                          \
    TESTING_CHECK_(va_ op vb_, fatal,                                               \
                   "expected " #a " " #op " " #b ", got " << va_ << " vs " << vb_); \
  } while (0)

#define EXPECT_TRUE(c) TESTING_CHECK_((c), false, "expected true: " #c)
#define EXPECT_FALSE(c) TESTING_CHECK_(!(c), false, "expected false: " #c)
#define ASSERT_TRUE(c) TESTING_CHECK_((c), true, "expected true: " #c)
#define ASSERT_FALSE(c) TESTING_CHECK_(!(c), true, "expected false: " #c)
#define EXPECT_EQ(a, b) TESTING_CMP_(a, b, ==, false)
#define EXPECT_NE(a, b) TESTING_CMP_(a, b, !=, false)
#define EXPECT_LT(a, b) TESTING_CMP_(a, b, <, false)
#define EXPECT_LE(a, b) TESTING_CMP_(a, b, <=, false)
#define EXPECT_GT(a, b) TESTING_CMP_(a, b, >, false)
#define EXPECT_GE(a, b) TESTING_CMP_(a, b, >=, false)
#define ASSERT_EQ(a, b) TESTING_CMP_(a, b, ==, true)
#define ASSERT_NE(a, b) TESTING_CMP_(a, b, !=, true)
#define ASSERT_LT(a, b) TESTING_CMP_(a, b, <, true)
#define ASSERT_LE(a, b) TESTING_CMP_(a, b, <=, true)
#define ASSERT_GT(a, b) TESTING_CMP_(a, b, >, true)
#define ASSERT_GE(a, b) TESTING_CMP_(a, b, >=, true)
#define EXPECT_NEAR(a, b, tol) \
  TESTING_CHECK_(std::fabs((a) - (b)) <= (tol), false, #a " !~ " #b << ": " << (a) << " vs " << (b))
#define EXPECT_STREQ(a, b) EXPECT_EQ(std::string(a), std::string(b))

#define EXPECT_THROW(stmt, exc)                                                     \
  do {                                                                              \
    bool caught_ = false;                                                           \
    try {                                                                           \
      stmt;                                                                         \
    } catch (const exc&) {                                                          \
      caught_ = true;                                                               \
    } catch (...) {                                                                 \
    }                                                                               \
    TESTING_CHECK_(caught_, false, "expected " #stmt " to throw " #exc);            \
  } while (0)
#define ASSERT_THROW(stmt, exc) EXPECT_THROW(stmt, exc)
#define EXPECT_NO_THROW(stmt)                                                       \
  do {                                                                              \
    try {                                                                           \
      stmt;                                                                         \
    } catch (const std::exception& e_) {                                            \
      TESTING_CHECK_(false, false, "unexpected exception from " #stmt ": " << e_.what()); \
    }                                                                               \
  } while (0)
#define EXPECT_DEATH(stmt, regex_unused) \
  TESTING_CHECK_(::testing::DiesInChild([&]() { stmt; }), false, "expected death: " #stmt)
#define ASSERT_DEATH(stmt, regex_unused) \
  TESTING_CHECK_(::testing::DiesInChild([&]() { stmt; }), true, "expected death: " #stmt)

#endif  // DMLC_TESTS_CPP_TESTING_H_
