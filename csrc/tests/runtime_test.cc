// Native unit tests of the C++ runtime. Ports of every reference gtest
// (base/message_test, base/range_partition_manager_test,
// server/util/{progress_tracker,pending_buffer}_test, server/map_storage_test,
// server/consistency/{bsp,ssp,asp}_model_test, server/server_thread_test,
// worker/kv_client_table_test, driver/{simple_id_mapper,worker_spec,engine}_test,
// comm/{sender,mailbox}_test) with identical expected values, plus the tests the reference
// lacked: checkpoint round trips in all three models, BSP/ASP CheckPoint not hanging,
// libsvm/dumper round trip, heartbeat failure detection. Ports are ephemeral (no races).
#include <array>
#include <atomic>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cstdio>
#include <fstream>

#include "../runtime/checkpoint.h"
#include "../runtime/async_server.h"
#include "../runtime/comm.h"
#include "../runtime/config.h"
#include "../runtime/engine.h"
#include "../runtime/fs.h"
#include "../runtime/io.h"
#include "../runtime/serialization.h"
#include "../runtime/shard_io.h"
#include "../runtime/server.h"
#include "../runtime/worker.h"
#include "minitest.h"

using namespace minips;

namespace {

int FreePort() {
  int fd = ::socket(AF_INET, SOCK_STREAM, 0);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  a.sin_port = 0;
  ::bind(fd, (sockaddr*)&a, sizeof(a));
  socklen_t len = sizeof(a);
  ::getsockname(fd, (sockaddr*)&a, &len);
  int port = ntohs(a.sin_port);
  ::close(fd);
  return port;
}

std::string TmpDir() {
  char tmpl[] = "/tmp/minips_test_XXXXXX";
  char* d = mkdtemp(tmpl);
  return std::string(d) + "/";
}

Message MakeMsg(Flag flag, int sender, int recver, int model = 0) {
  Message m;
  m.meta.flag = flag;
  m.meta.sender = sender;
  m.meta.recver = recver;
  m.meta.model_id = model;
  return m;
}

template <typename V>
Message KV(Flag flag, int sender, std::vector<Key> keys, std::vector<V> vals = {}) {
  Message m = MakeMsg(flag, sender, 0);
  m.AddData(SArray<Key>(keys));
  if (flag == Flag::kAdd) m.AddData(SArray<V>(vals));
  return m;
}

template <typename V>
V ReplyVal(const Message& m, size_t i = 0) {
  return SArray<V>(m.data[1])[i];
}

void ResetWorkers(AbstractModel* model, ThreadsafeQueue<Message>* q, std::vector<uint32_t> tids) {
  Message reset;
  reset.AddData(SArray<uint32_t>(tids));
  model->ResetWorker(reset);
  Message r;
  q->WaitAndPop(&r);
  EXPECT_EQ(r.meta.flag, Flag::kResetWorkerInModel);
}

}  // namespace

// ------------------------------------------------------------------------------ base
TEST(Message, AddData) {
  Message m;
  SArray<Key> keys({1, 2, 3});
  SArray<float> vals({0.1f, 0.2f, 0.3f});
  m.AddData(keys);
  m.AddData(vals);
  ASSERT_EQ(m.data.size(), 2u);
  EXPECT_EQ(SArray<Key>(m.data[0])[2], 3u);
  EXPECT_EQ(SArray<float>(m.data[1])[1], 0.2f);
  EXPECT_EQ(std::string(FlagName(Flag::kScaleRollback)), std::string("kScaleRollback"));
  EXPECT_EQ((int)Flag::kGet, 5);
}

TEST(SArray, SegmentZeroCopy) {
  SArray<int> a({1, 2, 3, 4, 5});
  auto s = a.segment(1, 4);
  EXPECT_EQ(s.size(), 3u);
  s[0] = 42;
  EXPECT_EQ(a[1], 42);
  SArray<char> bytes(a);
  EXPECT_EQ(bytes.size(), 20u);
  EXPECT_THROW(SArray<double>(SArray<char>(SArray<int>({1, 2, 3}))));
}

TEST(RangePartitionManager, SliceKeys) {
  RangePartitionManager pm({0, 1, 2}, {{2, 4}, {4, 7}, {7, 10}});
  SArray<Key> keys({2, 8, 9});
  std::vector<std::pair<int, Keys>> sliced;
  pm.Slice(keys, &sliced);
  ASSERT_EQ(sliced.size(), 2u);
  EXPECT_EQ(sliced[0].first, 0);
  EXPECT_EQ(sliced[1].first, 2);
  ASSERT_EQ(sliced[0].second.size(), 1u);
  ASSERT_EQ(sliced[1].second.size(), 2u);
  EXPECT_EQ(sliced[0].second[0], 2u);
  EXPECT_EQ(sliced[1].second[0], 8u);
  EXPECT_EQ(sliced[1].second[1], 9u);
}

TEST(RangePartitionManager, SliceKVs) {
  RangePartitionManager pm({0, 1, 2}, {{0, 4}, {4, 8}, {8, 10}});
  SArray<Key> keys({2, 5, 9});
  SArray<double> vals({.2, .5, .9});
  std::vector<std::pair<int, KVPairs>> sliced;
  pm.Slice(std::make_pair(keys, vals), &sliced);
  ASSERT_EQ(sliced.size(), 3u);
  for (int i = 0; i < 3; ++i) {
    EXPECT_EQ(sliced[i].first, i);
    ASSERT_EQ(sliced[i].second.first.size(), 1u);
    ASSERT_EQ(sliced[i].second.second.size(), 1u);
  }
  EXPECT_EQ(sliced[0].second.first[0], 2u);
  EXPECT_DOUBLE_EQ(sliced[1].second.second[0], .5);
  EXPECT_DOUBLE_EQ(sliced[2].second.second[0], .9);
}

TEST(RangePartitionManager, VectorValuedKeys) {
  RangePartitionManager pm({0, 1}, {{0, 2}, {2, 4}});
  SArray<Key> keys({1, 3});
  SArray<double> vals({1, 1, 3, 3});  // 2 values per key
  std::vector<std::pair<int, KVPairs>> sliced;
  pm.Slice(std::make_pair(keys, vals), &sliced);
  ASSERT_EQ(sliced.size(), 2u);
  EXPECT_EQ(sliced[1].second.second.size(), 2u);
  EXPECT_DOUBLE_EQ(sliced[1].second.second[0], 3);
}

TEST(EvenRanges, MatchesReferenceGetRanges) {
  auto r = EvenRanges(10, 3);
  ASSERT_EQ(r.size(), 3u);
  EXPECT_EQ(r[0].begin(), 0u);
  EXPECT_EQ(r[0].end(), 3u);
  EXPECT_EQ(r[2].begin(), 6u);
  EXPECT_EQ(r[2].end(), 10u);
}

TEST(Context, TypedFlags) {
  auto& ctx = Context::Get();
  ctx.ResetToDefaults();
  ctx.ParseArgs(std::vector<std::string>{"--my_id=3", "--checkpoint_toggle", "--num_dims", "100", "pos"});
  EXPECT_EQ(ctx.get_int32("my_id"), 3);
  EXPECT_TRUE(ctx.get_bool("checkpoint_toggle"));
  EXPECT_EQ(ctx.get_int64("num_dims"), 100);
  EXPECT_THROW(ctx.get_int32("no_such_flag"));
  EXPECT_THROW(ctx.set("my_id", std::string("abc")));
  EXPECT_THROW(ctx.ParseArgs(std::vector<std::string>{"--bogus=1"}));
  ctx.ResetToDefaults();
}

// ------------------------------------------------------------------------------ server utils
TEST(ProgressTracker, Init) {
  ProgressTracker p;
  p.Init({2, 4, 6});
  EXPECT_EQ(p.GetNumThreads(), 3);
  EXPECT_TRUE(p.CheckThreadValid(2));
  EXPECT_FALSE(p.CheckThreadValid(3));
  EXPECT_EQ(p.GetMinClock(), 0);
}

TEST(ProgressTracker, AdvanceAndGetChangedMinClock) {
  ProgressTracker p;
  p.Init({0, 1});
  EXPECT_EQ(p.AdvanceAndGetChangedMinClock(0), -1);  // [1,0]
  EXPECT_EQ(p.AdvanceAndGetChangedMinClock(1), 1);   // [1,1]
  EXPECT_EQ(p.AdvanceAndGetChangedMinClock(1), -1);  // [1,2]
  EXPECT_EQ(p.AdvanceAndGetChangedMinClock(1), -1);  // [1,3]
  EXPECT_EQ(p.AdvanceAndGetChangedMinClock(0), 2);   // [2,3]
  EXPECT_EQ(p.GetProgress(0), 2);
  EXPECT_EQ(p.GetProgress(1), 3);
  EXPECT_EQ(p.GetMinClock(), 2);
}

TEST(ProgressTracker, DeleteNodeAdvancesMin) {
  ProgressTracker p;
  p.Init({100, 1100});
  p.AdvanceAndGetChangedMinClock(100);
  EXPECT_EQ(p.DeleteNode(1), 1);  // node 1's tid was the unique min
  EXPECT_EQ(p.GetNumThreads(), 1);
}

TEST(ProgressTracker, DumpRestoreRoundTrip) {
  std::string dir = TmpDir();
  ProgressTracker p;
  p.Init({100, 101});
  for (int i = 0; i < 7; ++i) p.AdvanceAndGetChangedMinClock(100);
  for (int i = 0; i < 5; ++i) p.AdvanceAndGetChangedMinClock(101);
  p.Dump(dir + "prog", false);
  ProgressTracker q;
  q.Restore(dir + "prog");
  EXPECT_EQ(q.GetMinClock(), 5);
  EXPECT_EQ(q.GetProgress(100), 7);
  EXPECT_EQ(q.GetProgress(101), 5);
  EXPECT_EQ(ProgressTracker::RoundHundred(149), 100);
}

TEST(PendingBuffer, PushPop) {
  PendingBuffer b;
  b.Push(1, MakeMsg(Flag::kGet, 1, 0));
  b.Push(1, MakeMsg(Flag::kGet, 2, 0));
  b.Push(2, MakeMsg(Flag::kGet, 3, 0));
  EXPECT_EQ(b.Size(1), 2);
  EXPECT_EQ(b.Size(2), 1);
  auto v = b.Pop(1);
  EXPECT_EQ(v.size(), 2u);
  EXPECT_EQ(b.Size(1), 0);
  EXPECT_EQ(b.PopAll().size(), 1u);
  EXPECT_EQ(b.TotalSize(), 0);
}

TEST(MapStorage, AddGetInt) {
  MapStorage<int> s;
  s.Add(KV<int>(Flag::kAdd, 0, {0, 1}, {10, 20}));
  s.Add(KV<int>(Flag::kAdd, 0, {1}, {5}));
  Message r = s.Get(KV<int>(Flag::kGet, 7, {0, 1, 2}));
  EXPECT_EQ(r.meta.recver, 7);
  EXPECT_EQ(ReplyVal<int>(r, 0), 10);
  EXPECT_EQ(ReplyVal<int>(r, 1), 25);
  EXPECT_EQ(ReplyVal<int>(r, 2), 0);  // default-inserted
}

TEST(MapStorage, AddGetFloat) {
  MapStorage<float> s;
  s.SubAdd(SArray<Key>({3}), SArray<char>(SArray<float>({0.5f})));
  s.SubAdd(SArray<Key>({3}), SArray<char>(SArray<float>({0.25f})));
  SArray<float> v(s.SubGet(SArray<Key>({3})));
  EXPECT_EQ(v[0], 0.75f);
}

TEST(VectorStorage, DumpRestoreRoundTrip) {
  std::string dir = TmpDir();
  CheckpointConfig c;
  c.toggle = true;
  c.prefix = dir;
  c.my_id = 2;
  VectorStorage<double> s(Range(100, 110));
  s.SubAdd(SArray<Key>({101, 105, 109}), SArray<char>(SArray<double>({1.5, -2.25, 1e-9})));
  s.Dump(c);
  std::ifstream in(dir + "server_params_2");
  std::string line;
  std::getline(in, line);
  EXPECT_EQ(line.substr(0, 6), std::string("1:1.5 "));  // "<local_idx>:<val> " format
  VectorStorage<double> t(Range(100, 110));
  t.Restore(c);
  EXPECT_EQ(t.Data(), s.Data());
  EXPECT_THROW(t.SubGet(SArray<Key>({99})));
}

// ------------------------------------------------------------------------------ models
TEST(BSPModel, CheckGetAndAdd) {
  ThreadsafeQueue<Message> q;
  std::unique_ptr<AbstractStorage> st(new MapStorage<int>());
  BSPModel model(0, std::move(st), &q, CheckpointConfig());
  ResetWorkers(&model, &q, {2, 3});
  Message g0 = KV<int>(Flag::kGet, 2, {1});
  model.Get(g0);
  ASSERT_EQ(q.Size(), 1u);
  Message useless;
  q.WaitAndPop(&useless);
  Message m1 = KV<int>(Flag::kAdd, 2, {1}, {100});
  model.Add(m1);
  Message m2 = MakeMsg(Flag::kClock, 2, 0);
  model.Clock(m2);
  EXPECT_EQ(model.GetProgress(2), 1);
  EXPECT_EQ(model.GetProgress(3), 0);
  EXPECT_EQ(model.GetAddPendingSize(), 1);
  Message cm1 = KV<int>(Flag::kGet, 3, {1});
  model.Get(cm1);
  ASSERT_EQ(q.Size(), 1u);
  Message r1;
  q.WaitAndPop(&r1);
  EXPECT_EQ(ReplyVal<int>(r1), 0);  // add invisible until every worker clocks
  // A Get from the worker that already clocked waits for the superstep.
  Message early = KV<int>(Flag::kGet, 2, {1});
  model.Get(early);
  EXPECT_EQ(q.Size(), 0u);
  EXPECT_EQ(model.GetGetPendingSize(), 1);
  Message m3 = MakeMsg(Flag::kClock, 3, 0);
  model.Clock(m3);
  EXPECT_EQ(model.GetProgress(3), 1);
  EXPECT_EQ(model.GetAddPendingSize(), 0);
  ASSERT_EQ(q.Size(), 1u);
  Message r_early;
  q.WaitAndPop(&r_early);
  EXPECT_EQ(ReplyVal<int>(r_early), 100);
  Message cm2 = KV<int>(Flag::kGet, 3, {1});
  model.Get(cm2);
  Message r2;
  q.WaitAndPop(&r2);
  EXPECT_EQ(ReplyVal<int>(r2), 100);
}

TEST(SSPModel, CheckGetAndAdd) {
  ThreadsafeQueue<Message> q;
  std::unique_ptr<AbstractStorage> st(new MapStorage<int>());
  SSPModel model(0, std::move(st), 1, &q, CheckpointConfig());
  ResetWorkers(&model, &q, {2, 3});
  Message m3 = KV<int>(Flag::kAdd, 2, {0}, {1}), m4 = KV<int>(Flag::kAdd, 3, {1}, {2});
  Message m5 = KV<int>(Flag::kGet, 2, {0}), m6 = KV<int>(Flag::kGet, 3, {1});
  model.Add(m3);
  model.Add(m4);
  model.Get(m5);
  model.Get(m6);
  ASSERT_EQ(q.Size(), 2u);
  Message c;
  q.WaitAndPop(&c);
  EXPECT_EQ(SArray<Key>(c.data[0])[0], 0u);
  EXPECT_EQ(ReplyVal<int>(c), 1);
  EXPECT_EQ(c.meta.recver, 2);
  q.WaitAndPop(&c);
  EXPECT_EQ(SArray<Key>(c.data[0])[0], 1u);
  EXPECT_EQ(ReplyVal<int>(c), 2);
  EXPECT_EQ(c.meta.recver, 3);
}

TEST(SSPModel, CheckClock) {
  ThreadsafeQueue<Message> q;
  std::unique_ptr<AbstractStorage> st(new MapStorage<int>());
  SSPModel model(0, std::move(st), 1, &q, CheckpointConfig());
  ResetWorkers(&model, &q, {2, 3});
  Message a = MakeMsg(Flag::kClock, 2, 0), b = MakeMsg(Flag::kClock, 3, 0), c = MakeMsg(Flag::kClock, 2, 0);
  model.Clock(a);
  model.Clock(b);
  model.Clock(c);
  EXPECT_EQ(model.GetProgress(2), 2);
  EXPECT_EQ(model.GetProgress(3), 1);
}

TEST(SSPModel, CheckStaleness) {
  ThreadsafeQueue<Message> q;
  std::unique_ptr<AbstractStorage> st(new MapStorage<int>());
  SSPModel model(0, std::move(st), 2, &q, CheckpointConfig());
  ResetWorkers(&model, &q, {2, 3});
  Message g = KV<int>(Flag::kGet, 2, {0});
  model.Get(g);
  Message r;
  q.WaitAndPop(&r);
  Message c1 = MakeMsg(Flag::kClock, 2, 0);
  model.Clock(c1);
  Message a = KV<int>(Flag::kAdd, 2, {0}, {1});
  model.Add(a);
  Message c2 = MakeMsg(Flag::kClock, 2, 0), c3 = MakeMsg(Flag::kClock, 2, 0);
  model.Clock(c2);
  model.Clock(c3);  // worker 2 at progress 3, worker 3 at 0: 3 > 0 + 2
  EXPECT_EQ(model.GetProgress(2), 3);
  Message g2 = KV<int>(Flag::kGet, 2, {0});
  model.Get(g2);
  EXPECT_EQ(q.Size(), 0u);
  EXPECT_EQ(model.GetPendingSize(1), 1);  // parked under progress - staleness
  Message s1 = MakeMsg(Flag::kClock, 3, 0);
  model.Clock(s1);  // min clock -> 1 releases it
  ASSERT_EQ(q.Size(), 1u);
  q.WaitAndPop(&r);
  EXPECT_EQ(ReplyVal<int>(r), 1);
  EXPECT_EQ(model.GetPendingSize(1), 0);
}

TEST(ASPModel, NeverBlocks) {
  ThreadsafeQueue<Message> q;
  std::unique_ptr<AbstractStorage> st(new MapStorage<int>());
  ASPModel model(0, std::move(st), &q, CheckpointConfig());
  ResetWorkers(&model, &q, {2, 3});
  for (int i = 0; i < 5; ++i) {
    Message c = MakeMsg(Flag::kClock, 2, 0);
    model.Clock(c);
  }
  Message a = KV<int>(Flag::kAdd, 2, {0}, {7});
  model.Add(a);
  Message g = KV<int>(Flag::kGet, 2, {0});
  model.Get(g);
  ASSERT_EQ(q.Size(), 1u);
  Message r;
  q.WaitAndPop(&r);
  EXPECT_EQ(ReplyVal<int>(r), 7);
  EXPECT_EQ(model.GetProgress(2), 5);
  EXPECT_EQ(model.GetProgress(3), 0);
}

// Checkpoint round trip in all three models; every model answers kCheckpoint.
TEST(Models, CheckpointRoundTripAllModels) {
  for (int kind = 0; kind < 3; ++kind) {
    std::string dir = TmpDir();
    CheckpointConfig c;
    c.toggle = true;
    c.prefix = dir;
    c.my_id = 0;
    ThreadsafeQueue<Message> q;
    auto make = [&](std::unique_ptr<AbstractStorage> st) -> std::unique_ptr<ModelBase> {
      if (kind == 0) return std::unique_ptr<ModelBase>(new BSPModel(0, std::move(st), &q, c));
      if (kind == 1) return std::unique_ptr<ModelBase>(new SSPModel(0, std::move(st), 1, &q, c));
      return std::unique_ptr<ModelBase>(new ASPModel(0, std::move(st), &q, c));
    };
    auto model = make(std::unique_ptr<AbstractStorage>(new VectorStorage<double>(Range(0, 8))));
    ResetWorkers(model.get(), &q, {100});
    Message a = KV<double>(Flag::kAdd, 100, {1, 6}, {0.5, -3.0});
    model->Add(a);
    Message clk = MakeMsg(Flag::kClock, 100, 0);
    model->Clock(clk);
    Message ck = MakeMsg(Flag::kCheckpoint, 100, 0);
    model->Dump(ck);
    Message reply;
    ASSERT_TRUE(q.WaitAndPopFor(&reply, 1.0));  // reference BSP/ASP never replied (hang)
    EXPECT_EQ(reply.meta.flag, Flag::kCheckpoint);
    EXPECT_EQ(reply.meta.recver, 100);
    auto fresh = make(std::unique_ptr<AbstractStorage>(new VectorStorage<double>(Range(0, 8))));
    fresh->Restore();
    EXPECT_EQ(fresh->tracker().GetProgress(100), 1);
    auto* vs = dynamic_cast<VectorStorage<double>*>(fresh->storage());
    EXPECT_DOUBLE_EQ(vs->Data()[1], 0.5);
    EXPECT_DOUBLE_EQ(vs->Data()[6], -3.0);
  }
}

// ------------------------------------------------------------------------------ server thread
namespace {
class FakeModel : public AbstractModel {
 public:
  void Clock(Message&) override { clock++; }
  void Add(Message&) override { add++; }
  void Get(Message&) override { get++; }
  int GetProgress(int) override { return 0; }
  void ResetWorker(Message&) override { reset++; }
  void Dump(Message&) override {}
  void Restore() override {}
  void Update(int, const std::vector<Node>&, const Range&) override {}
  std::atomic<int> clock{0}, add{0}, get{0}, reset{0};
};
}  // namespace

TEST(ServerThread, Dispatch) {
  ServerThread st(0);
  auto* fm = new FakeModel();
  st.RegisterModel(0, std::unique_ptr<AbstractModel>(fm));
  st.Start();
  auto* q = st.GetWorkQueue();
  q->Push(MakeMsg(Flag::kClock, 1, 0));
  q->Push(MakeMsg(Flag::kAdd, 1, 0));
  q->Push(MakeMsg(Flag::kAdd, 1, 0));
  q->Push(MakeMsg(Flag::kGet, 1, 0));
  q->Push(MakeMsg(Flag::kResetWorkerInModel, 1, 0));
  q->Push(MakeMsg(Flag::kGet, 1, 0, /*model=*/9));  // unknown model: dropped
  st.Stop();
  EXPECT_EQ(fm->clock.load(), 1);
  EXPECT_EQ(fm->add.load(), 2);
  EXPECT_EQ(fm->get.load(), 1);
  EXPECT_EQ(fm->reset.load(), 1);
}

// ------------------------------------------------------------------------------ client table
namespace {
class FakePartitionManager : public AbstractPartitionManager {
 public:
  FakePartitionManager(const std::vector<uint32_t>& servers, Key split)
      : AbstractPartitionManager(servers), pm_(servers, {{0, split}, {split, 1u << 30}}) {}
  void Slice(const Keys& k, std::vector<std::pair<int, Keys>>* s) const override { pm_.Slice(k, s); }
  void Slice(const KVPairs& k, std::vector<std::pair<int, KVPairs>>* s) const override { pm_.Slice(k, s); }
  void SliceBytes(const Keys& k, const SArray<char>& v,
                  std::vector<std::tuple<int, Keys, SArray<char>>>* s) const override {
    pm_.SliceBytes(k, v, s);
  }
  void Update(const std::vector<Range>&, const std::vector<uint32_t>&) override {}

 private:
  RangePartitionManager pm_;
};
constexpr uint32_t kTestAppThreadId = 15;
constexpr uint32_t kTestModelId = 23;
}  // namespace

TEST(KVClientTable, Add) {
  ThreadsafeQueue<Message> queue;
  FakePartitionManager manager({0, 1}, 4);
  CallbackRunner cb;
  KVClientTable<double> table(kTestAppThreadId, kTestModelId, &queue, &manager, &cb);
  table.Add(std::vector<Key>{3, 4, 5, 6}, std::vector<double>{0.1, 0.1, 0.1, 0.1});
  Message m1, m2;
  queue.WaitAndPop(&m1);
  queue.WaitAndPop(&m2);
  EXPECT_EQ(m1.meta.sender, (int)kTestAppThreadId);
  EXPECT_EQ(m1.meta.recver, 0);
  EXPECT_EQ(m1.meta.model_id, (int)kTestModelId);
  EXPECT_EQ(m1.meta.flag, Flag::kAdd);
  ASSERT_EQ(m1.data.size(), 2u);
  EXPECT_EQ(SArray<Key>(m1.data[0]).size(), 1u);
  EXPECT_DOUBLE_EQ(SArray<double>(m1.data[1])[0], 0.1);
  EXPECT_EQ(m2.meta.recver, 1);
  ASSERT_EQ(SArray<Key>(m2.data[0]).size(), 3u);
  EXPECT_EQ(SArray<Key>(m2.data[0])[2], 6u);
}

TEST(KVClientTable, GetReassemblesInKeyOrder) {
  ThreadsafeQueue<Message> queue;
  FakePartitionManager manager({0, 1}, 4);
  CallbackRunner cb;
  std::vector<double> vals;
  std::thread th([&] {
    KVClientTable<double> table(kTestAppThreadId, kTestModelId, &queue, &manager, &cb);
    table.Get(std::vector<Key>{3, 4, 5, 6}, &vals);
  });
  Message m1, m2;
  queue.WaitAndPop(&m1);
  queue.WaitAndPop(&m2);
  EXPECT_EQ(m1.meta.flag, Flag::kGet);
  ASSERT_EQ(m1.data.size(), 1u);
  // Reply out of order: the second slice first.
  Message r2, r1;
  r2.AddData(SArray<Key>({4, 5, 6}));
  r2.AddData(SArray<double>({0.4, 0.2, 0.3}));
  r1.AddData(SArray<Key>({3}));
  r1.AddData(SArray<double>({0.1}));
  cb.AddResponse(kTestAppThreadId, kTestModelId, r2);
  cb.AddResponse(kTestAppThreadId, kTestModelId, r1);
  th.join();
  std::vector<double> expected{0.1, 0.4, 0.2, 0.3};
  EXPECT_TRUE(vals == expected);
}

// ------------------------------------------------------------------------------ driver
TEST(SimpleIdMapper, Init) {
  Node n1{0, "worker1", 12352}, n2{1, "worker1", 12353}, n3{3, "worker1", 12354};
  SimpleIdMapper m(n1, {n1, n2, n3});
  m.Init(1);
  EXPECT_EQ(m.GetServerThreadsForId(0).size(), 1u);
  EXPECT_EQ(m.GetServerThreadsForId(0)[0], 0u);
  EXPECT_EQ(m.GetWorkerHelperThreadsForId(0)[0], SimpleIdMapper::kWorkerHelperThreadId);
  EXPECT_EQ(m.GetServerThreadsForId(1)[0], SimpleIdMapper::kMaxThreadsPerNode);
  EXPECT_EQ(m.GetServerThreadsForId(3)[0], 3 * SimpleIdMapper::kMaxThreadsPerNode);
  EXPECT_EQ(m.GetWorkerHelperThreadsForId(3)[0],
            3 * SimpleIdMapper::kMaxThreadsPerNode + SimpleIdMapper::kWorkerHelperThreadId);
  EXPECT_EQ(m.GetNodeIdForThread(3 * SimpleIdMapper::kMaxThreadsPerNode + 1), 3u);
  EXPECT_EQ(m.GetNodeIdForThread(0), 0u);
}

TEST(SimpleIdMapper, AllocateDeallocateThread) {
  Node n1{0, "w", 1}, n2{1, "w", 2}, n3{3, "w", 3};
  SimpleIdMapper m(n1, {n1, n2, n3});
  m.Init(1);
  const uint32_t base = SimpleIdMapper::kMaxThreadsPerNode + SimpleIdMapper::kMaxBgThreadsPerNode;
  EXPECT_EQ(m.AllocateWorkerThread(1), base);
  EXPECT_EQ(m.AllocateWorkerThread(1), base + 1);
  EXPECT_EQ(m.GetWorkerThreadsForId(1).size(), 2u);
  m.DeallocateWorkerThread(1, base);
  EXPECT_EQ(m.GetWorkerThreadsForId(1).size(), 1u);
  EXPECT_EQ(m.GetWorkerThreadsForId(1)[0], base + 1);
  EXPECT_EQ(m.GetNodeIdForThread(base), 1u);
}

TEST(WorkerSpec, GetWorker) {
  WorkerSpec spec({{0, 3}, {1, 2}});
  EXPECT_TRUE(spec.HasLocalWorkers(0));
  ASSERT_EQ(spec.GetLocalWorkers(0).size(), 3u);
  ASSERT_EQ(spec.GetLocalWorkers(1).size(), 2u);
  EXPECT_EQ(spec.GetLocalWorkers(0)[0], 0u);
  EXPECT_EQ(spec.GetLocalWorkers(1)[1], 4u);
}

TEST(WorkerSpec, InsertWorkerIdThreadId) {
  WorkerSpec spec({{0, 3}, {1, 2}});
  const uint32_t bg = SimpleIdMapper::kMaxBgThreadsPerNode, tpn = SimpleIdMapper::kMaxThreadsPerNode;
  spec.InsertWorkerIdThreadId(0, bg);
  spec.InsertWorkerIdThreadId(1, bg + 1);
  spec.InsertWorkerIdThreadId(2, bg + 2);
  spec.InsertWorkerIdThreadId(3, tpn + bg);
  spec.InsertWorkerIdThreadId(4, tpn + bg + 1);
  EXPECT_EQ(spec.GetLocalThreads(0).size(), 3u);
  EXPECT_EQ(spec.GetLocalThreads(1)[1], tpn + bg + 1);
  auto all = spec.GetAllThreadIds();
  ASSERT_EQ(all.size(), 5u);
  EXPECT_EQ(all[3], tpn + bg);
  EXPECT_THROW(spec.InsertWorkerIdThreadId(0, 999));
}

// ------------------------------------------------------------------------------ comm
namespace {
class FakeMailbox : public AbstractMailbox {
 public:
  int Send(const Message& m) override {
    q.Push(m);
    return 0;
  }
  ThreadsafeQueue<Message> q;
};
class FakeIdMapper : public AbstractIdMapper {
 public:
  uint32_t GetNodeIdForThread(uint32_t tid) override { return tid; }
};
}  // namespace

TEST(Sender, ForwardsToMailbox) {
  FakeMailbox mb;
  Sender s(&mb);
  s.Start();
  for (int i = 0; i < 3; ++i) s.GetMessageQueue()->Push(MakeMsg(Flag::kGet, 0, i));
  s.Stop();
  EXPECT_EQ(mb.q.Size(), 3u);
  Message m;
  mb.q.WaitAndPop(&m);
  EXPECT_EQ(m.meta.recver, 0);
}

TEST(Mailbox, SendRecvTwoNodes) {
  Node n0{0, "localhost", FreePort()}, n1{1, "localhost", FreePort()};
  FakeIdMapper idm;
  Mailbox m0(n0, {n0, n1}, &idm), m1(n1, {n0, n1}, &idm);
  std::thread t0([&] { m0.Start(); });
  std::thread t1([&] { m1.Start(); });
  t0.join();
  t1.join();
  ThreadsafeQueue<Message> q0, q1;
  m0.RegisterQueue(0, &q0);
  m1.RegisterQueue(1, &q1);
  Message m = MakeMsg(Flag::kGet, 0, 1, 5);
  m.meta.failed_node_id = 9;
  m.AddData(SArray<Key>({1, 2, 3}));
  m0.Send(m);
  Message r;
  ASSERT_TRUE(q1.WaitAndPopFor(&r, 5));
  EXPECT_EQ(r.meta.sender, 0);
  EXPECT_EQ(r.meta.model_id, 5);
  EXPECT_EQ(r.meta.failed_node_id, 9);  // carried on the wire (reference dropped it)
  EXPECT_EQ(SArray<Key>(r.data[0])[2], 3u);
  m1.Send(MakeMsg(Flag::kAdd, 1, 0));  // reply direction
  ASSERT_TRUE(q0.WaitAndPopFor(&r, 5));
  m0.Send(MakeMsg(Flag::kClock, 0, 0));  // same-node fast path
  ASSERT_TRUE(q0.WaitAndPopFor(&r, 5));
  EXPECT_EQ(r.meta.flag, Flag::kClock);
  std::thread s0([&] { m0.Stop(); });
  std::thread s1([&] { m1.Stop(); });
  s0.join();
  s1.join();
}

TEST(Mailbox, BarrierFourNodes) {
  std::vector<Node> nodes;
  for (uint32_t i = 0; i < 4; ++i) nodes.push_back(Node{i, "localhost", FreePort()});
  FakeIdMapper idm;
  std::vector<std::unique_ptr<Mailbox>> mbs;
  for (auto& n : nodes) mbs.emplace_back(new Mailbox(n, nodes, &idm));
  std::vector<std::thread> th;
  for (auto& mb : mbs)
    th.emplace_back([&mb] {
      mb->Start();
      for (int r = 0; r < 10; ++r) mb->Barrier();
      mb->Stop();
    });
  for (auto& t : th) t.join();
  EXPECT_TRUE(true);
}

// ------------------------------------------------------------------------------ engine
TEST(Mailbox, BarrierTwoNodes) {
  // reference comm/mailbox_test.cpp:201-226 (ephemeral ports here, not fixed ones)
  std::vector<Node> nodes;
  for (uint32_t i = 0; i < 2; ++i) nodes.push_back(Node{i, "localhost", FreePort()});
  FakeIdMapper idm;
  std::atomic<int> passed{0};
  std::vector<std::unique_ptr<Mailbox>> mbs;
  for (auto& n : nodes) mbs.emplace_back(new Mailbox(n, nodes, &idm));
  std::vector<std::thread> th;
  for (auto& mb : mbs)
    th.emplace_back([&mb, &passed] {
      mb->Start();
      mb->Barrier();
      passed.fetch_add(1);
      mb->Barrier();
      // both nodes passed the first barrier before either leaves the second
      if (passed.load() != 2) throw std::runtime_error("barrier let a node through early");
      mb->Stop();
    });
  for (auto& t : th) t.join();
  EXPECT_EQ(passed.load(), 2);
}

TEST(Engine, SingleNodeMapStorageTask) {
  // reference driver/engine_test.cpp:51-92 (StartEverything on one node + SimpleTaskMapStorage)
  Context::Get().ResetToDefaults();
  Node me{0, "localhost", FreePort()};
  Engine engine(me, {me});
  engine.StartEverything(1);
  auto t = engine.CreateTable<double>(EvenRanges(100, 1), ModelType::ASP, StorageType::Map, 0);
  engine.Barrier();
  MLTask task;
  task.SetWorkerAlloc({{0, 4}});
  task.SetTables({t});
  std::atomic<int> ran{0};
  task.SetLambda([&](const Info& info) {
    auto table = info.CreateKVClientTable<double>(t);
    table->Add(std::vector<Key>{3, 97}, std::vector<double>{1.0, 2.0});
    table->Clock();
    ran.fetch_add(1);
  });
  engine.Run(task);
  std::vector<double> v;
  MLTask check;
  check.SetWorkerAlloc({{0, 1}});
  check.SetTables({t});
  check.SetLambda([&](const Info& info) {
    auto table = info.CreateKVClientTable<double>(t);
    table->Get(std::vector<Key>{3, 50, 97}, &v);
  });
  engine.Run(check);
  engine.StopEverything();
  EXPECT_EQ(ran.load(), 4);
  ASSERT_EQ(v.size(), 3u);
  EXPECT_DOUBLE_EQ(v[0], 4.0);
  EXPECT_DOUBLE_EQ(v[1], 0.0);  // MapStorage default for a never-added key
  EXPECT_DOUBLE_EQ(v[2], 8.0);
}

TEST(Engine, MultipleEnginesKVRoundTrip) {
  Context::Get().ResetToDefaults();
  std::vector<Node> nodes;
  for (uint32_t i = 0; i < 3; ++i) nodes.push_back(Node{i, "localhost", FreePort()});
  std::vector<double> results[3];
  auto run = [&](int id) {
    Engine engine(nodes[id], nodes);
    engine.StartEverything(1);
    auto t0 = engine.CreateTable<double>(EvenRanges(30, 3), ModelType::SSP, StorageType::Vector, 1);
    auto t1 = engine.CreateTable<double>(EvenRanges(30, 3), ModelType::BSP, StorageType::Map, 0);
    engine.Barrier();
    MLTask task;
    task.SetWorkerAlloc({{0, 3}, {1, 2}, {2, 3}});
    task.SetTables({t0, t1});
    std::mutex mu;
    task.SetLambda([&](const Info& info) {
      auto table = info.CreateKVClientTable<double>(t0);
      auto bsp = info.CreateKVClientTable<double>(t1);
      std::vector<Key> keys = {0, 5, 11, 29};
      for (int it = 0; it < 5; ++it) {
        std::vector<double> vals;
        table->Get(keys, &vals);
        table->Add(keys, std::vector<double>(4, 1.0));
        table->Clock();
        std::vector<double> bv;
        bsp->Get(keys, &bv);
        // BSP: every worker sees exactly `it` full supersteps of 8 workers' adds.
        if (bv[0] != 8.0 * it) throw std::runtime_error("BSP value mismatch");
        bsp->Add(keys, std::vector<double>(4, 1.0));
        bsp->Clock();
      }
      std::vector<double> vals;
      table->Get(keys, &vals);
      std::lock_guard<std::mutex> lk(mu);
      if (info.worker_id == 0) results[id] = vals;
    });
    engine.Run(task);
    // After Run's final barrier every add has been applied: 8 workers x 5 iterations.
    MLTask check;
    check.SetWorkerAlloc({{0, 1}});
    check.SetTables({t0});
    check.SetLambda([&](const Info& info) {
      auto table = info.CreateKVClientTable<double>(t0);
      std::vector<double> v;
      table->Get(std::vector<Key>{0, 29}, &v);
      results[0] = v;
    });
    engine.Run(check);
    engine.StopEverything();
  };
  std::vector<std::thread> th;
  for (int i = 0; i < 3; ++i) th.emplace_back(run, i);
  for (auto& t : th) t.join();
  ASSERT_EQ(results[0].size(), 2u);
  EXPECT_DOUBLE_EQ(results[0][0], 40.0);
  EXPECT_DOUBLE_EQ(results[0][1], 40.0);
}

TEST(Engine, CheckpointUnderBSPDoesNotHang) {
  Context::Get().ResetToDefaults();
  std::string dir = TmpDir();
  Context::Get().set("checkpoint_toggle", true);
  Context::Get().set("checkpoint_file_prefix", dir);
  Node n{0, "localhost", FreePort()};
  Engine engine(n, {n});
  engine.StartEverything(1);
  auto t = engine.CreateTable<double>(EvenRanges(10, 1), ModelType::BSP, StorageType::Vector);
  MLTask task;
  task.SetWorkerAlloc({{0, 1}});
  task.SetTables({t});
  task.SetLambda([&](const Info& info) {
    auto table = info.CreateKVClientTable<double>(t);
    table->Add(std::vector<Key>{3}, std::vector<double>{2.5});
    table->Clock();
    table->CheckPoint();
  });
  engine.Run(task);
  engine.StopEverything();
  std::ifstream in(dir + "server_params_0");
  std::string s;
  in >> s;
  EXPECT_EQ(s, std::string("3:2.5"));
  Context::Get().ResetToDefaults();
}

// ------------------------------------------------------------------------------ lib / io
TEST(Libsvm, ParseAndDumpRoundTrip) {
  SVMItem it;
  std::string line = "-1 3:0.5 10:2";
  ASSERT_TRUE(ParseLibsvm(line.data(), line.size(), &it));
  EXPECT_DOUBLE_EQ(it.y, -1);
  ASSERT_EQ(it.x.size(), 2u);
  EXPECT_EQ(it.x[0].first, 2);  // 1-based -> 0-based
  std::string dir = TmpDir();
  DumpSVMData(dir + "worker_0", {it, it});
  auto back = LoadSVMData(dir + "worker_0");
  ASSERT_EQ(back.size(), 2u);
  EXPECT_EQ(back[1].x[1].first, 9);  // no off-by-one on reload
  EXPECT_DOUBLE_EQ(back[1].x[1].second, 2);
  DumpConfigData(dir + "cfg", {{0, 300}, {1, 299}});
  auto cfg = LoadConfigData(dir + "cfg");
  EXPECT_EQ(cfg[1], 299);
}

TEST(Libsvm, ShardedLoad) {
  std::string dir = TmpDir();
  {
    std::ofstream out(dir + "data.svm");
    for (int i = 0; i < 100; ++i) out << (i % 2 ? 1 : -1) << " " << i + 1 << ":1\n";
  }
  size_t total = 0;
  for (int s = 0; s < 3; ++s) total += LoadLibsvmFile(dir + "data.svm", s, 3, 2).size();
  EXPECT_EQ(total, 100u);
}

TEST(BatchDataSampler, SortedUniqueKeys) {
  std::vector<SVMItem> data(3);
  data[0].x = {{5, 1}, {2, 1}};
  data[1].x = {{2, 1}, {9, 1}};
  data[2].x = {{1, 1}};
  BatchDataSampler s(&data, 2);
  auto k = s.PrepareNextBatch();
  std::vector<Key> e{2, 5, 9};
  EXPECT_TRUE(k == e);
  EXPECT_EQ(s.GetDataPtrs().size(), 2u);
}

TEST(Master, HeartbeatDetectsSilentNode) {
  Context::Get().ResetToDefaults();
  Context::Get().Define("heartbeat_interval_ms", Context::Type::kInt, "0");
  Context::Get().set("heartbeat_interval_ms", 50);
  Context::Get().set("heartbeat_interval", 1);
  Node master{1, "localhost", FreePort()};
  master.is_master = true;
  Node n0{0, "localhost", FreePort()}, n2{2, "localhost", FreePort()};
  Master m(master, {n0, n2});
  // Node 0 heartbeats, node 2 never does.
  Engine e0(n0, {n0}, master);
  e0.StartEverything(1);
  std::this_thread::sleep_for(std::chrono::milliseconds(600));
  auto det = m.GetCheckThread()->Detected();
  ASSERT_GE(det.size(), 1u);
  EXPECT_EQ(det[0], 2);
  e0.StopEverything();
  m.StopMaster();
  Context::Get().ResetToDefaults();
}

// ----------------------------------------------------------------------------- BinStream
struct Custom {
  int a = 0;
  std::string s;
  void serialize(minips::BinStream& b) const { b << a << s; }
  void deserialize(minips::BinStream& b) { b >> a >> s; }
};

TEST(BinStream, RoundTrip) {
  using namespace minips;
  BinStream b;
  std::vector<double> v{1.5, -2.0};
  std::map<int, std::string> m{{1, "x"}, {7, "yz"}};
  std::unordered_map<std::string, int> um{{"k", 3}};
  std::vector<std::string> vs{"a", "", "bcd"};
  SArray<Key> keys{3, 9, 27};
  auto sp = std::make_shared<int>(42);
  std::shared_ptr<int> nul;
  Custom c;
  c.a = 5;
  c.s = "hi";
  std::vector<Custom> vc{c, c};
  b << 7 << std::string("hello") << v << m << um << vs << keys << std::make_pair(1, 2.5) << sp << nul << c << vc;
  int i;
  std::string str;
  std::vector<double> v2;
  std::map<int, std::string> m2;
  std::unordered_map<std::string, int> um2;
  std::vector<std::string> vs2;
  SArray<Key> k2;
  std::pair<int, double> pr;
  std::shared_ptr<int> sp2, nul2 = std::make_shared<int>(1);
  Custom c2;
  std::vector<Custom> vc2;
  BinStream r = BinStream::FromSArray(b.ToSArray());
  r >> i >> str >> v2 >> m2 >> um2 >> vs2 >> k2 >> pr >> sp2 >> nul2 >> c2 >> vc2;
  EXPECT_EQ(i, 7);
  EXPECT_EQ(str, std::string("hello"));
  EXPECT_TRUE(v2 == v);
  EXPECT_TRUE(m2 == m);
  EXPECT_TRUE(um2 == um);
  EXPECT_TRUE(vs2 == vs);
  EXPECT_EQ(k2.size(), 3u);
  EXPECT_EQ(k2[2], (Key)27);
  EXPECT_EQ(pr.second, 2.5);
  EXPECT_EQ(*sp2, 42);
  EXPECT_TRUE(nul2 == nullptr);
  EXPECT_EQ(c2.s, std::string("hi"));
  EXPECT_EQ(vc2.size(), 2u);
  EXPECT_EQ(r.size(), 0u);
  EXPECT_THROW(r >> i);
}

// ----------------------------------------------------------------------------- shard files
TEST(ShardIO, BinaryAndTextRoundTrip) {
  using namespace minips;
  std::vector<float> params{0.f, 1.5f, 0.f, -2.25f, 3.f, 0.f};
  std::vector<float> state{0.1f, 0.2f, 0.3f};
  ShardMeta m;
  m.global_rows = 10;
  m.base = 4;
  m.rows = 3;
  m.cols = 2;
  m.clock = 17;
  m.table_id = 1;
  m.rank = 2;
  m.world = 3;
  m.kind = "sparse";
  const std::string dir = "/tmp/minips_shard_test_" + std::to_string(::getpid()) + "/";
  AsyncShardWriter w;
  auto t = w.Submit([&] {
    WriteShard(dir + "a.bin", m, {{"params", params.data(), DType::kF32, 3, 2}, {"state", state.data(),
                                                                                 DType::kF32, 3, 1}});
    WriteTextParams(dir + "a.txt", {"params", params.data(), DType::kF32, 3, 2});
  });
  w.Wait(t);
  EXPECT_EQ(w.TakeError(), std::string());
  LoadedShard s = ReadShard(dir + "a.bin");
  EXPECT_EQ(s.meta.clock, 17);
  EXPECT_EQ(s.meta.kind, std::string("sparse"));
  ASSERT_EQ(s.arrays.size(), 2u);
  EXPECT_EQ(std::memcmp(s.arrays[0].bytes.data(), params.data(), 24), 0);
  EXPECT_EQ(s.arrays[1].rows, 3u);
  auto txt = ReadTextParams(dir + "a.txt", 6);
  for (int i = 0; i < 6; ++i) EXPECT_EQ((float)txt[i], params[i]);
  std::ifstream raw(dir + "a.txt");
  std::string line;
  std::getline(raw, line);
  EXPECT_EQ(line, std::string("1:1.5 3:-2.25 4:3 "));
  EXPECT_THROW(ReadShard(dir + "a.txt"));
  auto t2 = w.Submit([] { throw std::runtime_error("disk full"); });
  w.Wait(t2);
  EXPECT_EQ(w.TakeError(), std::string("disk full"));
}

// ----------------------------------------------------------------------------- io
TEST(IO, LinesReadExactlyOnceAcrossBlocks) {
  using namespace minips;
  const std::string dir = "/tmp/minips_io_test_" + std::to_string(::getpid()) + "/";
  EnsureParentDir(dir + "x");
  uint64_t expect_sum = 0, expect_lines = 0;
  for (int f = 0; f < 3; ++f) {
    std::ofstream o(dir + "part-" + std::to_string(f));
    for (int i = 0; i < 257 + 31 * f; ++i) {
      const int v = f * 100000 + i;
      o << v << std::string((size_t)(i * 7 % 23), ' ') << "\n";
      expect_sum += (uint64_t)v;
      expect_lines++;
    }
    if (f == 2) o << 999999;  // last line without a trailing newline
  }
  expect_sum += 999999;
  expect_lines++;
  auto files = ListInputFiles(dir);
  ASSERT_EQ(files.size(), 3u);
  for (uint64_t bs : {1ull, 7ull, 64ull, 1000ull, 1ull << 20}) {
    for (int ranks : {1, 3}) {
      std::atomic<uint64_t> sum{0}, lines{0};
      for (int r = 0; r < ranks; ++r) {
        lines += LoadLines(files, bs, r, ranks, 4, [&](const char* l, size_t n, int) {
          sum += std::stoull(std::string(l, n));
        });
      }
      EXPECT_EQ(lines.load(), expect_lines);
      EXPECT_EQ(sum.load(), expect_sum);
    }
  }
}

TEST(IO, AsyncReadBufferKeepsOrder) {
  using namespace minips;
  int next = 0;
  AsyncReadBuffer<int> buf([&](int* out) {
    if (next >= 100) return false;
    *out = next++;
    return true;
  }, 4);
  int v, expect = 0;
  while (buf.Get(&v)) EXPECT_EQ(v, expect++);
  EXPECT_EQ(expect, 100);
}

TEST(IO, RemoteWindowReaderMatchesMmap) {
  // The buffered block window (remote file systems) yields exactly the lines of the mmap path.
  using namespace minips;
  const std::string path = "/tmp/minips_io_win_" + std::to_string(::getpid());
  {
    std::ofstream o(path);
    for (int i = 0; i < 3000; ++i) o << i << std::string((size_t)(i * 13 % 97), 'x') << "\n";
    o << "tail-without-newline";
  }
  MappedFile mf(path);
  auto rf = FileSystem::For(path).OpenRead(path);
  for (uint64_t bs : {1ull, 5ull, 333ull, 4096ull, 1ull << 22}) {
    std::vector<std::string> a, b;
    std::string win;
    for (auto& blk : SplitFiles({path}, bs)) {
      LineInputFormat x(mf, blk);
      LineInputFormat y = ReadBlockWindow(rf.get(), blk, &win);
      const char* l;
      size_t n;
      while (x.Next(&l, &n)) a.emplace_back(l, n);
      while (y.Next(&l, &n)) b.emplace_back(l, n);
    }
    EXPECT_EQ(a.size(), 3001u);
    EXPECT_TRUE(a == b);
  }
  ::unlink(path.c_str());
}

TEST(IO, LocalityAssignerPrefersLocalAndDropsReplicas) {
  using namespace minips;
  std::vector<FileBlock> blocks;
  // 6 blocks: 0-2 on {a,b}, 3-4 on {b,c}, 5 on {c}
  const std::vector<std::vector<std::string>> hosts = {{"a", "b"}, {"a", "b"}, {"a", "b"},
                                                       {"b", "c"}, {"b", "c"}, {"c"}};
  for (int i = 0; i < 6; ++i) blocks.push_back(FileBlock{"f", (uint64_t)i * 10, 10, 60, i, hosts[i]});
  LocalityAssigner a(blocks);
  std::vector<int> seen(6, 0);
  for (int i = 0; i < 3; ++i) {  // a gets its three local blocks
    auto b = a.Next("a");
    ASSERT_TRUE(b.has_value());
    EXPECT_TRUE(b->id <= 2);
    seen[b->id]++;
  }
  auto b = a.Next("b");  // a's blocks are gone from b's list too: b gets 3 or 4
  ASSERT_TRUE(b.has_value());
  EXPECT_TRUE(b->id == 3 || b->id == 4);
  seen[b->id]++;
  auto r = a.Next("a");  // nothing local left for a: a remote block (from c, which has the most)
  ASSERT_TRUE(r.has_value());
  EXPECT_TRUE(r->id >= 3);
  seen[r->id]++;
  while (auto x = a.Next("zz")) seen[x->id]++;
  for (int i = 0; i < 6; ++i) EXPECT_EQ(seen[i], 1);
  EXPECT_EQ(a.LocalServed(), 4u);
  EXPECT_EQ(a.RemoteServed(), 2u);
  EXPECT_FALSE(a.Next("a").has_value());
}

TEST(IO, AssignerServiceHandsEveryBlockOnce) {
  // node 0's assigner service + coordinated loaders of 3 "nodes" x 2 threads: every line is read
  // exactly once and the service halts after all 6 loader threads sent kExit.
  using namespace minips;
  const std::string dir = "/tmp/minips_io_asg_" + std::to_string(::getpid()) + "/";
  EnsureParentDir(dir + "x");
  uint64_t expect = 0;
  for (int f = 0; f < 4; ++f) {
    std::ofstream o(dir + "part-" + std::to_string(f));
    for (int i = 0; i < 500; ++i) {
      o << (f * 1000 + i) << "\n";
      expect += (uint64_t)(f * 1000 + i);
    }
  }
  BlockAssignerServer srv(0);
  srv.Start();
  std::atomic<uint64_t> sum{0}, lines{0};
  std::vector<std::thread> nodes;
  for (int r = 0; r < 3; ++r) {
    nodes.emplace_back([&, r] {
      LoadOptions opt;
      opt.rank = r;
      opt.num_ranks = 3;
      opt.num_threads = 2;
      opt.block_size = 512;
      opt.assigner = "127.0.0.1:" + std::to_string(srv.Port());
      opt.host = "host" + std::to_string(r);
      lines += ForEachLine(dir, opt, [&](const FileBlock&, const char* l, size_t n, int) {
        sum += std::stoull(std::string(l, n));
      });
    });
  }
  for (auto& t : nodes) t.join();
  EXPECT_TRUE(srv.WaitDone(10));
  srv.Stop();
  EXPECT_EQ(lines.load(), 2000u);
  EXPECT_EQ(sum.load(), expect);
  // local files: every block is "on" this host, which none of the fake hosts is -> all remote
  EXPECT_EQ(srv.LocalServed(), 0u);
  EXPECT_TRUE(srv.RemoteServed() > 0);
}

TEST(FS, UrlsAndGeneralStreams) {
  using namespace minips;
  Url u = ParseUrl("hdfs://nn.example:9000/data/a.txt");
  EXPECT_EQ(u.scheme, std::string("hdfs"));
  EXPECT_EQ(u.host, std::string("nn.example"));
  EXPECT_EQ(u.port, 9000);
  EXPECT_EQ(u.path, std::string("/data/a.txt"));
  Url w = ParseUrl("http://dn1:9864/webhdfs/v1/x?op=OPEN&offset=3");
  EXPECT_EQ(w.query, std::string("op=OPEN&offset=3"));
  EXPECT_EQ(ParseUrl("/tmp/x").scheme, std::string(""));
  EXPECT_EQ(ParseUrl("file:///tmp/x").path, std::string("/tmp/x"));
  EXPECT_TRUE(IsLocalUrl("file:///tmp/x"));
  EXPECT_FALSE(IsLocalUrl("webhdfs://nn:9870/x"));
  const std::string p = "file:///tmp/minips_fs_" + std::to_string(::getpid());
  {
    GeneralOfstream o(p);
    for (int i = 0; i < 200000; ++i) o << i << " ";
    o.close();
    EXPECT_TRUE(o.good());
  }
  GeneralIfstream in(p);
  int v, expect = 0;
  while (in >> v) EXPECT_EQ(v, expect++);
  EXPECT_EQ(expect, 200000);
  GeneralIfstream s(p);
  s.seekg(6);  // "0 1 2 3 " -> token at byte 6 is "3"
  s >> v;
  EXPECT_EQ(v, 3);
  GeneralIfstream missing("/nonexistent/minips/file");
  EXPECT_FALSE(missing.good());
  std::string why;
  if (!LibHdfs3Available(&why)) EXPECT_TRUE(why.find("webhdfs://") != std::string::npos);
  ::unlink(ParseUrl(p).path.c_str());
}

TEST(PSBoard, SspGateWakesOnAppliedAndTimesOut) {
  // Two ranks' views of one segment (as two processes map it). Rank 1 (an owner) applies rank 0's
  // and its own clocks one by one; rank 0's SSP gate (min applied >= 3) returns only after the
  // last publish, and a stuck owner makes the wait report a timeout instead of hanging.
  using namespace minips;
  const std::string name = "minips_psb_test_" + std::to_string(::getpid());
  PSBoard r0(name, 2, 0, 2), r1(name, 2, 1, 2);
  r0.PublishSent(1, 5);
  EXPECT_EQ(r1.Sent(1, 0), 5);
  EXPECT_EQ(r1.Sent(0, 0), 0);  // tables are independent
  EXPECT_EQ(r0.MinSent(1), 0);
  r0.PublishAppliedRow(1, 3);  // owner 0 has every requester's clocks < 3 of table 1
  EXPECT_EQ(r1.Applied(1, 0, 1), 3);
  EXPECT_EQ(r1.MinApplied(1), 0);
  std::atomic<int> published{0};
  std::thread owner([&] {
    for (int c = 1; c <= 3; ++c) {
      std::this_thread::sleep_for(std::chrono::milliseconds(20));
      published = c;
      r1.PublishApplied(1, 0, c);
      r1.PublishApplied(1, 1, c);
    }
  });
  const double waited = r0.WaitMinApplied(1, 3, 10.0);
  EXPECT_EQ(published.load(), 3);
  EXPECT_TRUE(waited > 0.03);
  EXPECT_EQ(r0.MinApplied(1), 3);
  EXPECT_EQ(r0.MinAppliedFrom(1, 0), 3);
  EXPECT_EQ(r0.OwnerVersion(1, 1), 6);
  owner.join();
  EXPECT_TRUE(r0.WaitMinApplied(1, 9, 0.05) < 0);  // timeout: reported, not thrown
  EXPECT_EQ(r1.Pending(1), 2);                      // rank 0 sent 5 clocks, owner 1 applied 3
  std::vector<int64_t> a = r0.SnapshotApplied(1);
  EXPECT_EQ(a.size(), 4u);
  EXPECT_EQ(a[0 * 2 + 1], 3);
  r0.Unlink();
}

namespace {
struct RecordingApplier : minips::Applier {
  std::vector<std::array<int64_t, 3>> seen;
  int flushes = 0;
  void Apply(int t, int r, int64_t c) override { seen.push_back({t, r, c}); }
  void Flush() override { ++flushes; }
};
}  // namespace

TEST(AsyncServer, AppliesArrivedClocksInOrderAndPauses) {
  // The owner-side server thread: every (table, requester, clock) that arrived is applied exactly
  // once, clock-major with the requesters interleaved, then published as applied; a paused
  // server applies nothing until resumed.
  using namespace minips;
  const std::string name = "minips_srv_test_" + std::to_string(::getpid());
  PSBoard req0(name, 2, 0, 2), req1(name, 2, 1, 2);
  RecordingApplier ap;
  AsyncServer srv(name, 2, 0, 2, &ap);
  srv.SetLog(true);
  srv.Enable(0);
  srv.Start();
  req1.PublishAppliedRow(0, 1000);  // owner 1 (no server in this test) has applied everything
  req0.PublishSent(0, 2);
  req1.PublishSent(0, 2);
  EXPECT_TRUE(req0.WaitAppliedFrom(0, 0, 2, 5.0) >= 0);
  EXPECT_TRUE(req1.WaitAppliedFrom(0, 1, 2, 5.0) >= 0);
  srv.Pause();
  req1.PublishSent(0, 3);
  std::this_thread::sleep_for(std::chrono::milliseconds(30));
  EXPECT_EQ(req1.Applied(0, 0, 1), 2);  // paused: clock 2 of requester 1 waits
  srv.Resume();
  EXPECT_TRUE(req1.WaitAppliedFrom(0, 1, 3, 5.0) >= 0);
  srv.Stop();
  EXPECT_EQ(srv.Error(), "");
  std::vector<int64_t> log = srv.TakeLog();
  EXPECT_EQ(log.size(), 15u);  // 5 applies
  EXPECT_EQ(srv.Applied(), 5);
  // the first wake-up saw both requesters at clock 2 (or applied them as they came): every
  // requester's clocks appear in increasing order
  int64_t last[2] = {-1, -1};
  for (size_t i = 0; i < log.size(); i += 3) {
    EXPECT_EQ(log[i], 0);
    EXPECT_TRUE(log[i + 2] == last[log[i + 1]] + 1);
    last[log[i + 1]] = log[i + 2];
  }
  EXPECT_TRUE(ap.flushes >= 1);
  req0.Unlink();
}

namespace {
struct ClockApplier : minips::Applier {
  std::vector<std::array<int64_t, 3>> seen;  // (table, requester or -1 = whole clock, clock)
  void Apply(int t, int r, int64_t c) override { seen.push_back({t, r, c}); }
  void ApplyClock(int t, int64_t c, int /*world*/) override { seen.push_back({t, -1, c}); }
  void Flush() override {}
};
}  // namespace

TEST(AsyncServer, CoalescedTableAppliesWholeClocksOnly) {
  // An SSP table served clock-coalesced (AsyncServer::SetCoalesce): clock c is applied once, as
  // one ApplyClock, only after EVERY requester sent it, and published for all requesters together;
  // a plain table of the same server keeps applying push by push.
  using namespace minips;
  const std::string name = "minips_srv_coal_" + std::to_string(::getpid());
  PSBoard req0(name, 2, 0, 2), req1(name, 2, 1, 2);
  ClockApplier ap;
  AsyncServer srv(name, 2, 0, 2, &ap);
  srv.SetCoalesce(0, true);
  srv.Enable(0);
  srv.Enable(1);
  srv.Start();
  req1.PublishAppliedRow(0, 1000);  // owner 1 (no server here) has applied everything
  req1.PublishAppliedRow(1, 1000);
  req0.PublishSent(0, 3);  // requester 0 ran ahead: clocks 0..2
  req0.PublishSent(1, 3);
  EXPECT_TRUE(req0.WaitAppliedFrom(1, 0, 3, 5.0) >= 0);  // the plain table applied them at once
  std::this_thread::sleep_for(std::chrono::milliseconds(30));
  EXPECT_EQ(req0.Applied(0, 0, 0), 0);  // coalesced: nothing until requester 1 sent clock 0
  req1.PublishSent(0, 2);               // requester 1: clocks 0..1
  EXPECT_TRUE(req0.WaitAppliedFrom(0, 0, 2, 5.0) >= 0);
  std::this_thread::sleep_for(std::chrono::milliseconds(30));
  EXPECT_EQ(req0.Applied(0, 0, 0), 2);  // clock 2 waits for requester 1 although requester 0 sent it
  EXPECT_EQ(req0.Applied(0, 0, 1), 2);  // published for both requesters together
  req1.PublishSent(0, 3);
  EXPECT_TRUE(req0.WaitAppliedFrom(0, 1, 3, 5.0) >= 0);
  srv.Stop();
  EXPECT_EQ(srv.Error(), "");
  std::vector<int64_t> want_clocks;
  for (const auto& e : ap.seen)
    if (e[0] == 0) {
      EXPECT_EQ(e[1], -1);  // table 0 only ever sees whole-clock applies
      want_clocks.push_back(e[2]);
    } else {
      EXPECT_TRUE(e[1] == 0);  // table 1: requester 0's pushes, one by one
    }
  EXPECT_EQ(want_clocks.size(), 3u);
  for (size_t i = 0; i < want_clocks.size(); ++i) EXPECT_EQ(want_clocks[i], (int64_t)i);
  req0.Unlink();
}

TEST(ShardIO, ReadsVersion1Files) {
  // Round-1 shard files (v1: each array's bytes right after its descriptor, no offsets) still
  // restore through the v2 reader (header parse + offset ranged reads).
  using namespace minips;
  const std::string path = "/tmp/minips_v1_" + std::to_string(::getpid()) + ".bin";
  {
    std::ofstream o(path, std::ios::binary);
    auto put = [&](const auto& v) { o.write(reinterpret_cast<const char*>(&v), sizeof(v)); };
    auto put_s = [&](const std::string& str) {
      put((uint32_t)str.size());
      o.write(str.data(), (std::streamsize)str.size());
    };
    o.write("MPSSHRD1", 8);
    put((uint32_t)1);
    put((uint64_t)10);  // global_rows
    put((uint64_t)4);   // base
    put((uint64_t)3);   // rows
    put((uint64_t)2);   // cols
    put((int64_t)7);    // clock
    put((int32_t)0);
    put((int32_t)1);
    put((int32_t)2);
    put_s("sparse");
    put((uint32_t)2);
    const float p[6] = {1, 2, 3, 4, 5, 6};
    put_s("params");
    put((uint32_t)DType::kF32);
    put((uint64_t)3);
    put((uint64_t)2);
    put((uint64_t)24);
    o.write(reinterpret_cast<const char*>(p), 24);
    const float st[3] = {0.5f, 0.25f, 0.125f};
    put_s("state");
    put((uint32_t)DType::kF32);
    put((uint64_t)3);
    put((uint64_t)1);
    put((uint64_t)12);
    o.write(reinterpret_cast<const char*>(st), 12);
  }
  LoadedShard s = ReadShard(path);
  EXPECT_EQ(s.meta.clock, 7);
  EXPECT_EQ(s.meta.base, 4u);
  EXPECT_EQ(s.arrays.size(), 2u);
  const float* got = reinterpret_cast<const float*>(s.arrays[0].bytes.data());
  EXPECT_EQ(got[5], 6.f);
  const float* gs = reinterpret_cast<const float*>(s.arrays[1].bytes.data());
  EXPECT_EQ(gs[2], 0.125f);
  float row[2];
  ReadRows(path, ReadShardHeader(path).arrays[0].offset, 8, 1, 1, row);  // partial (owner-range) read
  EXPECT_EQ(row[0], 3.f);
  ::unlink(path.c_str());
}

int main(int argc, char** argv) { return minitest::RunAll(argc, argv); }
