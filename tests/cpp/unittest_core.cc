// L0/L1 unit tests: the behaviours pinned by the reference's
// test/unittest/unittest_{any,array_view,config,env,json,logging,optional,
// param,serializer}.cc, re-expressed for this implementation.
#include <dmlc/any.h>
#include <dmlc/array_view.h>
#include <dmlc/common.h>
#include <dmlc/config.h>
#include <dmlc/json.h>
#include <dmlc/logging.h>
#include <dmlc/memory_io.h>
#include <dmlc/optional.h>
#include <dmlc/parameter.h>
#include <dmlc/registry.h>
#include <dmlc/serializer.h>
#include <dmlc/timer.h>

#include <cstdlib>
#include <list>
#include <map>
#include <set>
#include <sstream>
#include <string>
#include <unordered_map>
#include <vector>

#include "./testing.h"

// ---------------------------------------------------------------- any
TEST(Any, BasicsAndCopy) {
  dmlc::any a = std::string("hello");
  EXPECT_FALSE(a.empty());
  EXPECT_EQ(dmlc::get<std::string>(a), "hello");
  dmlc::any b = a;
  dmlc::get<std::string>(b) += "!";
  EXPECT_EQ(dmlc::get<std::string>(a), "hello");
  EXPECT_EQ(dmlc::get<std::string>(b), "hello!");
  dmlc::any c = std::move(b);
  EXPECT_EQ(dmlc::get<std::string>(c), "hello!");
  c.clear();
  EXPECT_TRUE(c.empty());
  dmlc::any v;
  v.construct<std::vector<int>>(3, 7);
  EXPECT_EQ(dmlc::get<std::vector<int>>(v).size(), 3U);
  EXPECT_THROW(dmlc::get<int>(a), dmlc::Error);
}

TEST(Any, DestroysHeldObject) {
  static int live = 0;
  struct Counted {
    Counted() { ++live; }
    Counted(const Counted&) { ++live; }
    ~Counted() { --live; }
  };
  {
    dmlc::any a = Counted();
    dmlc::any b = a;
    EXPECT_EQ(live, 2);
  }
  EXPECT_EQ(live, 0);
}

DMLC_JSON_ENABLE_ANY(int, int);
DMLC_JSON_ENABLE_ANY(std::string, str);
DMLC_JSON_ENABLE_ANY(std::vector<int>, vec_int);

TEST(Any, JsonRoundTrip) {
  std::unordered_map<std::string, dmlc::any> m;
  m["a"] = 3;
  m["b"] = std::string("text");
  m["c"] = std::vector<int>{1, 2, 3};
  std::ostringstream os;
  {
    dmlc::JSONWriter w(&os);
    w.Write(m);
  }
  std::istringstream is(os.str());
  dmlc::JSONReader r(&is);
  std::unordered_map<std::string, dmlc::any> back;
  r.Read(&back);
  EXPECT_EQ(dmlc::get<int>(back["a"]), 3);
  EXPECT_EQ(dmlc::get<std::string>(back["b"]), "text");
  EXPECT_EQ(dmlc::get<std::vector<int>>(back["c"])[2], 3);
}

// ---------------------------------------------------------------- array_view
TEST(ArrayView, VectorAndRange) {
  std::vector<int> v{1, 2, 3, 4};
  dmlc::array_view<int> a(v);
  EXPECT_EQ(a.size(), 4U);
  int sum = 0;
  for (int x : a) sum += x;
  EXPECT_EQ(sum, 10);
  dmlc::array_view<int> b(v.data() + 1, v.data() + 3);
  EXPECT_EQ(b.size(), 2U);
  EXPECT_EQ(b[1], 3);
}

// ---------------------------------------------------------------- common
TEST(Common, SplitAndHash) {
  auto parts = dmlc::Split("a,b,,c", ',');
  ASSERT_EQ(parts.size(), 4U);
  EXPECT_EQ(parts[3], "c");
  EXPECT_NE(dmlc::HashCombine(1, 2), dmlc::HashCombine(2, 1));
  EXPECT_GT(dmlc::GetTime(), 0.0);
}

// ---------------------------------------------------------------- config
TEST(Config, QuotesCommentsAndOrder) {
  std::istringstream is(
      "k1 = 1\n"
      "k2 = \"a string with \\\"quotes\\\" # not a comment\"\n"
      "# full line comment\n"
      "k3 = 3 # trailing\n"
      "k1 = 10\n");
  dmlc::Config single(is, false);
  EXPECT_EQ(single.GetParam("k1"), "10");
  EXPECT_EQ(single.GetParam("k2"), "a string with \"quotes\" # not a comment");
  EXPECT_TRUE(single.IsGenuineString("k2"));
  EXPECT_FALSE(single.IsGenuineString("k3"));
  std::vector<std::string> keys;
  for (auto kv : single) keys.push_back(kv.first);
  ASSERT_EQ(keys.size(), 3U);
  EXPECT_EQ(keys[0], "k2");  // k1 was overridden: it moves to its last position
  EXPECT_EQ(keys[2], "k1");

  std::istringstream is2("k = 1\nk = 2\nj = x\n");
  dmlc::Config multi(is2, true);
  std::vector<std::string> vals;
  for (auto kv : multi) {
    if (kv.first == "k") vals.push_back(kv.second);
  }
  ASSERT_EQ(vals.size(), 2U);
  EXPECT_EQ(vals[0], "1");
  EXPECT_EQ(multi.GetParam("k"), "2");
  multi.SetParam("n", 5);
  multi.SetParam("s", std::string("str"), true);
  std::string proto = multi.ToProtoString();
  EXPECT_TRUE(proto.find("n : 5") != std::string::npos);
  EXPECT_TRUE(proto.find("s : \"str\"") != std::string::npos);
}

// ---------------------------------------------------------------- env
TEST(Env, DefaultsForUnsetAndBlank) {
  unsetenv("DMLC_TEST_ENV_UNSET");
  EXPECT_EQ(dmlc::GetEnv("DMLC_TEST_ENV_UNSET", 42), 42);
  setenv("DMLC_TEST_ENV_BLANK", "", 1);
  EXPECT_EQ(dmlc::GetEnv("DMLC_TEST_ENV_BLANK", std::string("dflt")), "dflt");
  dmlc::SetEnv("DMLC_TEST_ENV_SET", 7);
  EXPECT_EQ(dmlc::GetEnv("DMLC_TEST_ENV_SET", 0), 7);
}

// ---------------------------------------------------------------- json
struct JsonThing {
  int a{0};
  std::string b;
  std::vector<float> c;
  int opt{-1};
  void Save(dmlc::JSONWriter* w) const {
    w->BeginObject();
    w->WriteObjectKeyValue("a", a);
    w->WriteObjectKeyValue("b", b);
    w->WriteObjectKeyValue("c", c);
    w->EndObject();
  }
  void Load(dmlc::JSONReader* r) {
    dmlc::JSONObjectReadHelper h;
    h.DeclareField("a", &a);
    h.DeclareField("b", &b);
    h.DeclareField("c", &c);
    h.DeclareOptionalField("opt", &opt);
    h.ReadAllFields(r);
  }
};

template <typename T>
static T JsonRoundTrip(const T& v) {
  std::ostringstream os;
  dmlc::JSONWriter w(&os);
  w.Write(v);
  std::istringstream is(os.str());
  dmlc::JSONReader r(&is);
  T out;
  r.Read(&out);
  return out;
}

TEST(Json, StlRoundTrips) {
  std::vector<int> v{1, -2, 3};
  EXPECT_TRUE(JsonRoundTrip(v) == v);
  std::vector<std::vector<double>> vv{{1.5}, {}, {2, 3}};
  EXPECT_TRUE(JsonRoundTrip(vv) == vv);
  std::map<std::string, int> m{{"x", 1}, {"y", 2}};
  EXPECT_TRUE(JsonRoundTrip(m) == m);
  std::unordered_map<std::string, std::vector<int>> um{{"k", {4, 5}}};
  EXPECT_TRUE(JsonRoundTrip(um) == um);
  std::list<std::string> l{"a\n\"b\"", "\t\\"};
  EXPECT_TRUE(JsonRoundTrip(l) == l);
  std::pair<std::string, int> p{"p", 9};
  EXPECT_TRUE(JsonRoundTrip(p) == p);
}

TEST(Json, ObjectHelperOptionalFields) {
  JsonThing t;
  t.a = 5;
  t.b = "bee";
  t.c = {0.5f, 2.0f};
  JsonThing back = JsonRoundTrip(t);
  EXPECT_EQ(back.a, 5);
  EXPECT_EQ(back.b, "bee");
  EXPECT_EQ(back.c.size(), 2U);
  EXPECT_EQ(back.opt, -1);  // optional field absent
  std::istringstream missing("{\"a\": 1, \"b\": \"x\"}");
  dmlc::JSONReader r(&missing);
  JsonThing bad;
  EXPECT_THROW(bad.Load(&r), dmlc::Error);  // required field c missing
}

// ---------------------------------------------------------------- logging
static void FailCheckInNoexcept(int x, int y) noexcept { CHECK_NE(x, y); }

TEST(Logging, CheckThrowsAndDies) {
  EXPECT_THROW(CHECK_EQ(1, 2) << "boom", dmlc::Error);
  EXPECT_THROW(LOG(FATAL) << "fatal", dmlc::Error);
  try {
    CHECK_LT(5, 3) << "context";
  } catch (const dmlc::Error& e) {
    EXPECT_TRUE(std::string(e.what()).find("context") != std::string::npos);
  }
  // an uncaught fatal error terminates the process (the reference's
  // ASSERT_DEATH with DMLC_LOG_FATAL_THROW=0)
  EXPECT_DEATH(FailCheckInNoexcept(1, 1), "");
}

// ---------------------------------------------------------------- optional
TEST(Optional, PrintParse) {
  dmlc::optional<int> x;
  std::ostringstream os;
  os << x;
  EXPECT_EQ(os.str(), "None");
  x = 5;
  std::ostringstream os2;
  os2 << x;
  EXPECT_EQ(os2.str(), "5");
  std::istringstream is("None 1L 7");
  dmlc::optional<int> a, b, c;
  is >> a >> b >> c;
  EXPECT_FALSE(a.has_value());
  EXPECT_EQ(*b, 1);
  EXPECT_EQ(*c, 7);
  std::istringstream bs("true false 1 0 none");
  dmlc::optional<bool> t, f, one, zero, none;
  bs >> t >> f >> one >> zero >> none;
  EXPECT_TRUE(*t);
  EXPECT_FALSE(*f);
  EXPECT_TRUE(*one);
  EXPECT_FALSE(*zero);
  EXPECT_FALSE(none.has_value());
}

// ---------------------------------------------------------------- parameter
struct TestParam : public dmlc::Parameter<TestParam> {
  float lr;
  int nthread;
  std::string name;
  int mode;
  dmlc::optional<int> maybe;
  dmlc::optional<bool> flag;
  DMLC_DECLARE_PARAMETER(TestParam) {
    DMLC_DECLARE_FIELD(lr).set_default(0.01f).set_range(0.0f, 10.0f).describe("learning rate");
    DMLC_DECLARE_FIELD(nthread).set_lower_bound(1).set_default(4);
    DMLC_DECLARE_FIELD(name).describe("required name");
    DMLC_DECLARE_FIELD(mode).add_enum("fast", 0).add_enum("exact", 1).set_default(0);
    DMLC_DECLARE_FIELD(maybe).add_enum("auto", -1).set_default(dmlc::optional<int>());
    DMLC_DECLARE_FIELD(flag).set_default(dmlc::optional<bool>());
    DMLC_DECLARE_ALIAS(lr, eta);
  }
};
DMLC_REGISTER_PARAMETER(TestParam);

TEST(Parameter, InitDefaultsAliasesEnums) {
  TestParam p;
  std::map<std::string, std::string> kw{{"name", "x"}, {"eta", "0.5"}, {"mode", "exact"},
                                        {"maybe", "auto"}, {"flag", "true"}};
  p.Init(kw);
  EXPECT_EQ(p.name, "x");
  EXPECT_NEAR(p.lr, 0.5f, 1e-7);
  EXPECT_EQ(p.nthread, 4);
  EXPECT_EQ(p.mode, 1);
  EXPECT_EQ(*p.maybe, -1);
  EXPECT_TRUE(*p.flag);
  auto dict = p.__DICT__();
  EXPECT_EQ(dict["mode"], "exact");
  EXPECT_EQ(dict["maybe"], "auto");
  EXPECT_TRUE(TestParam::__DOC__().find("learning rate") != std::string::npos);
}

TEST(Parameter, Errors) {
  TestParam p;
  EXPECT_THROW(p.Init(std::map<std::string, std::string>{}), dmlc::ParamError);  // name
  EXPECT_THROW(p.Init(std::map<std::string, std::string>{{"name", "x"}, {"lr", "11"}}),
               dmlc::ParamError);
  EXPECT_THROW(p.Init(std::map<std::string, std::string>{{"name", "x"}, {"nthread", "0"}}),
               dmlc::ParamError);
  EXPECT_THROW(p.Init(std::map<std::string, std::string>{{"name", "x"}, {"mode", "bogus"}}),
               dmlc::ParamError);
  EXPECT_THROW(p.Init(std::map<std::string, std::string>{{"name", "x"}, {"unknown", "1"}}),
               dmlc::ParamError);
  // reference unittest_param.cc: a denormal float is out of range for stof
  EXPECT_THROW(p.Init(std::map<std::string, std::string>{{"name", "x"}, {"lr", "9.4e-39"}}),
               dmlc::ParamError);
  auto unknown = p.InitAllowUnknown(
      std::map<std::string, std::string>{{"name", "y"}, {"other", "1"}});
  ASSERT_EQ(unknown.size(), 1U);
  EXPECT_EQ(unknown[0].first, "other");
  // hidden keys (__k__) are skipped by the default kAllowHidden option
  EXPECT_NO_THROW(p.Init(std::map<std::string, std::string>{{"name", "x"}, {"__hidden__", "1"}}));
}

TEST(Parameter, JsonSaveLoad) {
  TestParam p;
  p.Init(std::map<std::string, std::string>{{"name", "n"}, {"nthread", "8"}});
  std::ostringstream os;
  dmlc::JSONWriter w(&os);
  p.Save(&w);
  std::istringstream is(os.str());
  dmlc::JSONReader r(&is);
  TestParam q;
  q.Load(&r);
  EXPECT_EQ(q.nthread, 8);
  EXPECT_EQ(q.name, "n");
}

// ---------------------------------------------------------------- serializer
struct SaveLoadThing {
  int x{0};
  std::string s;
  void Save(dmlc::Stream* fo) const {
    fo->Write(x);
    fo->Write(s);
  }
  bool Load(dmlc::Stream* fi) { return fi->Read(&x) && fi->Read(&s); }
};

template <typename T>
static T BinaryRoundTrip(const T& v) {
  std::string buf;
  dmlc::MemoryStringStream ms(&buf);
  ms.Write(v);
  ms.Seek(0);
  T out;
  bool ok = ms.Read(&out);
  EXPECT_TRUE(ok);
  return out;
}

TEST(Serializer, StlComposites) {
  std::vector<int> v{1, 2, 3};
  EXPECT_TRUE(BinaryRoundTrip(v) == v);
  std::vector<std::string> vs{"a", "", "ccc"};
  EXPECT_TRUE(BinaryRoundTrip(vs) == vs);
  std::map<std::string, std::vector<double>> m{{"k", {1.0, 2.0}}, {"e", {}}};
  EXPECT_TRUE(BinaryRoundTrip(m) == m);
  std::set<int> st{5, 1, 3};
  EXPECT_TRUE(BinaryRoundTrip(st) == st);
  std::list<std::pair<int, std::string>> l{{1, "x"}, {2, "y"}};
  EXPECT_TRUE(BinaryRoundTrip(l) == l);
  std::unordered_map<int, std::string> um{{1, "one"}};
  EXPECT_TRUE(BinaryRoundTrip(um) == um);
  std::vector<SaveLoadThing> things(2);
  things[1].x = 7;
  things[1].s = "seven";
  auto back = BinaryRoundTrip(things);
  EXPECT_EQ(back[1].x, 7);
  EXPECT_EQ(back[1].s, "seven");
}

TEST(Serializer, PodVectorWireFormat) {
  // u64 count followed by raw elements (reference serializer.h:105-124)
  std::vector<uint32_t> v{0xdeadbeef, 7};
  std::string buf;
  dmlc::MemoryStringStream ms(&buf);
  ms.Write(v);
  ASSERT_EQ(buf.size(), 8U + 8U);
  uint64_t n;
  std::memcpy(&n, buf.data(), 8);
  EXPECT_EQ(n, 2U);
  uint32_t first;
  std::memcpy(&first, buf.data() + 8, 4);
  EXPECT_EQ(first, 0xdeadbeefU);
  // a truncated stream fails the read
  std::string cut = buf.substr(0, 10);
  dmlc::MemoryStringStream ms2(&cut);
  std::vector<uint32_t> out;
  EXPECT_FALSE(ms2.Read(&out));
}

// ---------------------------------------------------------------- registry
struct TestFactory : public dmlc::FunctionRegEntryBase<TestFactory, std::function<int(int)>> {};
DMLC_REGISTRY_ENABLE(TestFactory);
DMLC_REGISTRY_REGISTER(TestFactory, TestFactory, twice)
    .describe("double it")
    .set_body([](int x) { return 2 * x; });
DMLC_REGISTRY_REGISTER(TestFactory, TestFactory, square).set_body([](int x) { return x * x; });

TEST(Registry, FindAliasList) {
  auto* e = dmlc::Registry<TestFactory>::Find("twice");
  ASSERT_TRUE(e != nullptr);
  EXPECT_EQ(e->body(21), 42);
  EXPECT_EQ(e->description, "double it");
  dmlc::Registry<TestFactory>::Get()->AddAlias("square", "sq");
  EXPECT_EQ(dmlc::Registry<TestFactory>::Find("sq")->body(5), 25);
  EXPECT_TRUE(dmlc::Registry<TestFactory>::Find("nope") == nullptr);
  EXPECT_EQ(dmlc::Registry<TestFactory>::List().size(), 2U);
  EXPECT_EQ(dmlc::Registry<TestFactory>::ListAllNames().size(), 3U);  // names include aliases
}

// ------------------------------------------------- parameter / json (round 3)
TEST(Parameter, UpdateOptionalBoolAndDocs) {
  TestParam p;
  p.Init(std::map<std::string, std::string>{{"name", "a"}, {"nthread", "6"}});
  // UpdateAllowUnknown touches only the given fields and applies no defaults
  auto rest = p.UpdateAllowUnknown(
      std::map<std::string, std::string>{{"lr", "0.25"}, {"zzz", "1"}});
  ASSERT_EQ(rest.size(), 1U);
  EXPECT_EQ(rest[0].first, "zzz");
  EXPECT_EQ(p.nthread, 6);
  EXPECT_NEAR(p.lr, 0.25f, 1e-7);
  // optional<int> with enums: "None" empties it and prints back as None
  p.Init(std::map<std::string, std::string>{{"name", "a"}, {"maybe", "None"}, {"flag", " FALSE"}});
  EXPECT_FALSE(p.maybe.has_value());
  const auto dict = p.__DICT__();  // the EXPECT macros bind references: keep the map alive
  EXPECT_EQ(dict.at("maybe"), "None");
  EXPECT_FALSE(*p.flag);
  // trailing garbage after a number is an error; trailing blanks are not
  EXPECT_THROW(p.Init(std::map<std::string, std::string>{{"name", "a"}, {"nthread", "3x"}}),
               dmlc::ParamError);
  EXPECT_NO_THROW(p.Init(std::map<std::string, std::string>{{"name", "a"}, {"nthread", "3 "}}));
  EXPECT_EQ(p.nthread, 3);
  // field docs: required vs default, enum listing
  auto fields = TestParam::__FIELDS__();
  ASSERT_EQ(fields.size(), 6U);
  EXPECT_EQ(fields[2].name, "name");
  EXPECT_TRUE(fields[2].type_info_str.find("required") != std::string::npos);
  EXPECT_TRUE(fields[3].type_info_str.find("'exact'") != std::string::npos);
  EXPECT_TRUE(fields[3].type_info_str.find("default=fast") != std::string::npos);
  // kAllMatch rejects hidden keys too
  EXPECT_THROW(p.Init(std::map<std::string, std::string>{{"name", "a"}, {"__h__", "1"}},
                      dmlc::kAllMatch),
               dmlc::ParamError);
}

TEST(Json, WriterLayoutAndReaderErrors) {
  std::ostringstream os;
  dmlc::JSONWriter w(&os);
  std::map<std::string, std::vector<int>> m{{"a", {1, 2}}, {"b", {}}};
  w.Write(m);
  EXPECT_EQ(os.str(), "{\n  \"a\": [1, 2],\n  \"b\": []\n}");
  std::ostringstream os2;
  dmlc::JSONWriter w2(&os2);
  std::vector<std::map<std::string, int>> vm{{{"k", 1}}};
  w2.Write(vm);
  EXPECT_EQ(os2.str(), "[\n  {\n    \"k\": 1\n  }\n]");
  // \u escapes decode to UTF-8, a missing comma is an error
  std::istringstream is("[\"\\u00e9\\u0041\"]");
  dmlc::JSONReader r(&is);
  std::vector<std::string> v;
  r.Read(&v);
  ASSERT_EQ(v.size(), 1U);
  EXPECT_EQ(v[0], "\xc3\xa9" "A");
  std::istringstream bad("[1 2]");
  dmlc::JSONReader rb(&bad);
  std::vector<int> vi;
  EXPECT_THROW(rb.Read(&vi), dmlc::Error);
}
