// pybind11 bindings of the C++ PS runtime (module minips_amd._runtime).
// Blocking calls (Get, CheckPoint, Barrier, Run, Stop) release the GIL; worker lambdas
// passed to Engine.run are invoked on C++ threads that re-acquire it.
#include <pybind11/functional.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "../runtime/async_server.h"
#include "../runtime/checkpoint.h"
#include "../runtime/fs.h"
#include "../runtime/io.h"
#include "../runtime/comm.h"
#include "../runtime/config.h"
#include "../runtime/engine.h"
#include "../runtime/ps_board.h"
#include "../runtime/shard_io.h"

namespace py = pybind11;
using namespace minips;

namespace {

DType ParseDType(const std::string& s) {
  if (s == "float32") return DType::kF32;
  if (s == "bfloat16") return DType::kBF16;
  if (s == "float64") return DType::kF64;
  if (s == "int64") return DType::kI64;
  if (s == "int32") return DType::kI32;
  throw std::invalid_argument("unsupported dtype " + s);
}
const char* DTypeName(DType t) {
  switch (t) {
    case DType::kF32:
      return "float32";
    case DType::kBF16:
      return "bfloat16";
    case DType::kF64:
      return "float64";
    case DType::kI64:
      return "int64";
    case DType::kI32:
      return "int32";
  }
  return "?";
}
ShardMeta MetaFromDict(const py::dict& d) {
  ShardMeta m;
  m.global_rows = d["global_rows"].cast<uint64_t>();
  m.base = d["base"].cast<uint64_t>();
  m.rows = d["rows"].cast<uint64_t>();
  m.cols = d["cols"].cast<uint64_t>();
  m.clock = d["clock"].cast<int64_t>();
  m.table_id = d["table_id"].cast<int32_t>();
  m.rank = d["rank"].cast<int32_t>();
  m.world = d["world"].cast<int32_t>();
  m.kind = d["kind"].cast<std::string>();
  return m;
}
// arrays: [(name, data_ptr, dtype, rows, cols)] -- host memory kept alive by the caller
std::vector<ArrayRef> ArraysFromList(const py::list& l) {
  std::vector<ArrayRef> out;
  for (auto item : l) {
    auto t = item.cast<py::tuple>();
    ArrayRef a;
    a.name = t[0].cast<std::string>();
    a.data = reinterpret_cast<const void*>(t[1].cast<uintptr_t>());
    a.dtype = ParseDType(t[2].cast<std::string>());
    a.rows = t[3].cast<uint64_t>();
    a.cols = t[4].cast<uint64_t>();
    out.push_back(a);
  }
  return out;
}

template <typename Val>
void BindTable(py::module& m, const char* name) {
  py::class_<KVClientTable<Val>>(m, name)
      .def(
          "get",
          [](KVClientTable<Val>& t, py::array_t<uint64_t, py::array::c_style | py::array::forcecast> keys) {
            std::vector<Key> k(keys.data(), keys.data() + keys.size());
            std::vector<Val> vals;
            {
              py::gil_scoped_release rel;
              t.Get(k, &vals);
            }
            return py::array_t<Val>(vals.size(), vals.data());
          },
          "Blocking pull of sorted keys; returns values in key order.")
      .def(
          "add",
          [](KVClientTable<Val>& t, py::array_t<uint64_t, py::array::c_style | py::array::forcecast> keys,
             py::array_t<Val, py::array::c_style | py::array::forcecast> vals) {
            std::vector<Key> k(keys.data(), keys.data() + keys.size());
            std::vector<Val> v(vals.data(), vals.data() + vals.size());
            t.Add(k, v);
          },
          "Asynchronous push of (sorted keys, values).")
      .def("clock", &KVClientTable<Val>::Clock)
      .def("checkpoint", &KVClientTable<Val>::CheckPoint, py::call_guard<py::gil_scoped_release>())
      .def("heartbeat", &KVClientTable<Val>::HeartBeat, py::arg("node_id"), py::arg("quit") = false);
}

// The owner side of the asynchronous PS on a CPU rank (gloo tests): the same server loop as the
// GPU ranks (csrc/runtime/async_server.h), applying through a Python callable apply(t, r, c)
// that runs the table's CPU optimizer on the inbox slot. Exceptions become the server's error.
class PyApplier : public Applier {
 public:
  explicit PyApplier(py::function fn) : fn_(std::move(fn)) {}
  ~PyApplier() override {
    py::gil_scoped_acquire g;
    fn_ = py::function();
  }
  void Apply(int t, int r, int64_t c) override {
    py::gil_scoped_acquire g;
    try {
      fn_(t, r, c);
    } catch (py::error_already_set& e) {
      throw std::runtime_error(std::string("async server apply: ") + e.what());
    }
  }
  // a clock-coalesced table: apply(t, -1, c) applies every requester's slot of clock c at once
  void ApplyClock(int t, int64_t c, int /*world*/) override { Apply(t, -1, c); }
  void Flush() override {}
  // the owner's write lock of the table on the board (the CPU twin of the GPU lock words)
  void BeginTable(int t) override {
    if (board_ && !board_->WriteLock(t, 30.0)) throw std::runtime_error("async server: write lock timed out");
  }
  void EndTable(int t) override {
    if (board_) board_->WriteUnlock(t);
  }
  PSBoard* board_ = nullptr;

 private:
  py::function fn_;
};

class CpuAsyncServer {
 public:
  CpuAsyncServer(const std::string& board, int world, int rank, int tables, py::function apply)
      : applier_(std::move(apply)), server_(board, world, rank, tables, &applier_) {
    applier_.board_ = &server_.board();
  }
  ~CpuAsyncServer() {
    py::gil_scoped_release rel;
    server_.Stop();
  }
  AsyncServer& server() { return server_; }

 private:
  PyApplier applier_;
  AsyncServer server_;
};

}  // namespace

PYBIND11_MODULE(_runtime, m) {
  m.doc() = "minips_amd C++ parameter-server runtime";

  py::enum_<Flag>(m, "Flag")
      .value("kExit", Flag::kExit)
      .value("kBarrier", Flag::kBarrier)
      .value("kResetWorkerInModel", Flag::kResetWorkerInModel)
      .value("kClock", Flag::kClock)
      .value("kAdd", Flag::kAdd)
      .value("kGet", Flag::kGet)
      .value("kForceQuit", Flag::kForceQuit)
      .value("kCheckpoint", Flag::kCheckpoint)
      .value("kHeartBeat", Flag::kHeartBeat)
      .value("kQuitHeartBeat", Flag::kQuitHeartBeat)
      .value("kRollBack", Flag::kRollBack)
      .value("kScale", Flag::kScale)
      .value("kScaleRollback", Flag::kScaleRollback);
  py::enum_<ModelType>(m, "ModelType").value("SSP", ModelType::SSP).value("BSP", ModelType::BSP).value("ASP",
      ModelType::ASP);
  py::enum_<StorageType>(m, "StorageType").value("Map", StorageType::Map).value("Vector", StorageType::Vector);

  py::class_<Node>(m, "Node")
      .def(py::init([](uint32_t id, std::string host, int port, bool is_master, int gpu) {
             Node n;
             n.id = id;
             n.hostname = host;
             n.port = port;
             n.is_master = is_master;
             n.gpu = gpu;
             return n;
           }),
           py::arg("id") = 0, py::arg("hostname") = "localhost", py::arg("port") = 0, py::arg("is_master") = false,
           py::arg("gpu") = -1)
      .def_readwrite("id", &Node::id)
      .def_readwrite("hostname", &Node::hostname)
      .def_readwrite("port", &Node::port)
      .def_readwrite("is_master", &Node::is_master)
      .def_readwrite("gpu", &Node::gpu)
      .def("__repr__", &Node::DebugString);
  m.def("parse_file", &ParseFile);
  m.def("select_master", [](std::vector<Node> nodes, int hb) {
    Node master = SelectMaster(nodes, hb);
    return py::make_tuple(master, nodes);
  });
  m.def("check_valid_node_ids", &CheckValidNodeIds);
  m.def("check_consecutive_ids", &CheckConsecutiveIds);

  py::class_<Range>(m, "Range")
      .def(py::init<uint64_t, uint64_t>())
      .def("begin", &Range::begin)
      .def("end", &Range::end)
      .def("size", &Range::size)
      .def("__repr__", [](const Range& r) { return "[" + std::to_string(r.begin()) + ","
                                                     + std::to_string(r.end()) + ")"; });
  m.def("even_ranges", &EvenRanges);

  // --- Context (typed flag registry) --------------------------------------------------
  py::class_<Context, std::unique_ptr<Context, py::nodelete>>(m, "Context")
      .def_static("get", &Context::Get, py::return_value_policy::reference)
      .def("define",
           [](Context& c, const std::string& name, const std::string& type, const std::string& def,
              const std::string& help) {
             Context::Type t = type == "int" ? Context::Type::kInt
                               : type == "bool" ? Context::Type::kBool
                               : type == "double" ? Context::Type::kDouble
                                                  : Context::Type::kString;
             c.Define(name, t, def, help);
           },
           py::arg("name"), py::arg("type"), py::arg("default"), py::arg("help") = "")
      .def("has", &Context::Has)
      .def("get_string", &Context::get_string)
      .def("get_int32", &Context::get_int32)
      .def("get_int64", &Context::get_int64)
      .def("get_bool", &Context::get_bool)
      .def("get_double", &Context::get_double)
      .def("set", [](Context& c, const std::string& n, const std::string& v) { c.set(n, v); })
      .def("set_int", [](Context& c, const std::string& n, int64_t v) { c.set(n, v); })
      .def("set_bool", [](Context& c, const std::string& n, bool v) { c.set(n, v); })
      .def("parse_args", [](Context& c, const std::vector<std::string>& a, bool u) { return c.ParseArgs(a, u); },
           py::arg("args"), py::arg("allow_unknown") = false)
      .def("snapshot", &Context::Snapshot)
      .def("help", &Context::Help)
      .def("reset", &Context::ResetToDefaults)
      .def("set_iteration", &Context::SetIteration)
      .def("get_iteration", &Context::GetIteration)
      .def("iteration_map", &Context::GetIterationMap)
      .def("set_iteration_map", &Context::SetIterationMap);

  // --- consistency building blocks -----------------------------------------------------
  py::class_<ProgressTracker>(m, "ProgressTracker")
      .def(py::init<>())
      .def("init", &ProgressTracker::Init)
      .def("advance_and_get_changed_min_clock", &ProgressTracker::AdvanceAndGetChangedMinClock)
      .def("get_progress", &ProgressTracker::GetProgress)
      .def("get_min_clock", &ProgressTracker::GetMinClock)
      .def("get_num_threads", &ProgressTracker::GetNumThreads)
      .def("is_unique_min", &ProgressTracker::IsUniqueMin)
      .def("check_thread_valid", &ProgressTracker::CheckThreadValid)
      .def("delete_node", &ProgressTracker::DeleteNode)
      .def("dump", &ProgressTracker::Dump, py::arg("path"), py::arg("round_hundred") = false)
      .def("restore", &ProgressTracker::Restore, py::arg("path"), py::arg("scale_node_id") = -1)
      .def("progresses", &ProgressTracker::Progresses)
      .def("__repr__", &ProgressTracker::DebugString);

  py::class_<SimpleIdMapper>(m, "SimpleIdMapper")
      .def(py::init<Node, std::vector<Node>>())
      .def("init", &SimpleIdMapper::Init, py::arg("num_server_threads_per_node"), py::arg("skip_node_id") = -1)
      .def("get_node_id_for_thread", &SimpleIdMapper::GetNodeIdForThread)
      .def("allocate_worker_thread", &SimpleIdMapper::AllocateWorkerThread)
      .def("deallocate_worker_thread", &SimpleIdMapper::DeallocateWorkerThread)
      .def("get_server_threads_for_id", &SimpleIdMapper::GetServerThreadsForId)
      .def("get_worker_helper_threads_for_id", &SimpleIdMapper::GetWorkerHelperThreadsForId)
      .def("get_worker_threads_for_id", &SimpleIdMapper::GetWorkerThreadsForId)
      .def("get_all_server_threads", &SimpleIdMapper::GetAllServerThreads);
  m.attr("kMaxThreadsPerNode") = SimpleIdMapper::kMaxThreadsPerNode;
  m.attr("kMaxBgThreadsPerNode") = SimpleIdMapper::kMaxBgThreadsPerNode;
  m.attr("kWorkerHelperThreadId") = SimpleIdMapper::kWorkerHelperThreadId;

  py::class_<WorkerAlloc>(m, "WorkerAlloc")
      .def(py::init([](uint32_t node, uint32_t n) { return WorkerAlloc{node, n}; }))
      .def_readwrite("node_id", &WorkerAlloc::node_id)
      .def_readwrite("num_workers", &WorkerAlloc::num_workers);
  py::class_<WorkerSpec>(m, "WorkerSpec")
      .def(py::init<const std::vector<WorkerAlloc>&>())
      .def("has_local_workers", &WorkerSpec::HasLocalWorkers)
      .def("get_local_workers", &WorkerSpec::GetLocalWorkers)
      .def("get_local_threads", &WorkerSpec::GetLocalThreads)
      .def("get_all_thread_ids", &WorkerSpec::GetAllThreadIds)
      .def("insert_worker_id_thread_id", &WorkerSpec::InsertWorkerIdThreadId)
      .def("get_num_workers", &WorkerSpec::GetNumWorkers);

  py::class_<RangePartitionManager>(m, "RangePartitionManager")
      .def(py::init<const std::vector<uint32_t>&, const std::vector<Range>&, int>(), py::arg("server_thread_ids"),
           py::arg("ranges"), py::arg("master_node_id") = -1)
      .def("slice", [](const RangePartitionManager& pm, py::array_t<uint64_t,
                       py::array::c_style | py::array::forcecast> keys) {
        SArray<Key> k(keys.data(), keys.size());
        std::vector<std::pair<int, Keys>> sliced;
        pm.Slice(k, &sliced);
        py::list out;
        for (auto& s : sliced) out.append(py::make_tuple(s.first, py::array_t<uint64_t>(s.second.size(),
                                                                                        s.second.data())));
        return out;
      })
      .def("get_ranges", &RangePartitionManager::GetRanges);

  // --- engine / task / tables ----------------------------------------------------------
  py::class_<Info>(m, "Info")
      .def_readonly("thread_id", &Info::thread_id)
      .def_readonly("worker_id", &Info::worker_id)
      .def_readonly("node_id", &Info::node_id)
      .def("create_kv_client_table",
           [](const Info& info, uint32_t table_id, const std::string& dtype) -> py::object {
             if (dtype == "float32") return py::cast(info.CreateKVClientTable<float>(table_id).release(),
                                                     py::return_value_policy::take_ownership);
             return py::cast(info.CreateKVClientTable<double>(table_id).release(),
                             py::return_value_policy::take_ownership);
           },
           py::arg("table_id"), py::arg("dtype") = "float64");
  BindTable<double>(m, "KVClientTableF64");
  BindTable<float>(m, "KVClientTableF32");

  py::class_<MLTask>(m, "MLTask")
      .def(py::init<>())
      .def("set_lambda", &MLTask::SetLambda)
      .def("set_worker_alloc", &MLTask::SetWorkerAlloc)
      .def("set_tables", &MLTask::SetTables)
      .def("is_setup", &MLTask::IsSetup);

  py::class_<Engine>(m, "Engine")
      .def(py::init<const Node&, const std::vector<Node>&, const Node&, const Node&>(), py::arg("node"),
           py::arg("nodes"), py::arg("master") = Node(), py::arg("scale_node") = Node())
      .def("start_everything", &Engine::StartEverything, py::arg("num_server_threads_per_node") = 1,
           py::call_guard<py::gil_scoped_release>())
      .def("stop_everything", &Engine::StopEverything, py::call_guard<py::gil_scoped_release>())
      .def("barrier", &Engine::Barrier, py::call_guard<py::gil_scoped_release>())
      .def("force_quit", &Engine::ForceQuit)
      .def("run", &Engine::Run, py::call_guard<py::gil_scoped_release>())
      .def("get_ranges", &Engine::getRanges)
      .def(
          "create_table",
          [](Engine& e, const std::vector<Range>& ranges, ModelType mt, StorageType st, int staleness,
             const std::string& dtype) {
            if (dtype == "float32") return e.CreateTable<float>(ranges, mt, st, staleness);
            return e.CreateTable<double>(ranges, mt, st, staleness);
          },
          py::arg("ranges"), py::arg("model_type") = ModelType::BSP, py::arg("storage_type") = StorageType::Vector,
          py::arg("staleness") = 0, py::arg("dtype") = "float64")
      .def("set_dump_callback", &Engine::SetDumpCallback)
      .def("is_need_rollback", &Engine::IsNeedRollBack)
      .def("inc_rollback_count", &Engine::IncRollBackCount)
      .def("recover_end", &Engine::RecoverEnd)
      .def("wait_recover", &Engine::WaitRecover, py::call_guard<py::gil_scoped_release>())
      .def("rollback_count", &Engine::RollBackCount)
      .def("num_tables", &Engine::NumTables)
      .def("get_node", &Engine::GetNode)
      .def("get_nodes", &Engine::GetNodes)
      .def("bytes_sent", [](Engine& e) { return e.GetMailbox() ? e.GetMailbox()->BytesSent() : 0; });

  py::class_<Master>(m, "Master")
      .def(py::init<const Node&, const std::vector<Node>&>(), py::call_guard<py::gil_scoped_release>())
      .def("wait_all_quit", &Master::WaitAllQuit, py::arg("timeout_s") = 0.0, py::call_guard<py::gil_scoped_release>())
      .def("stop_master", &Master::StopMaster, py::call_guard<py::gil_scoped_release>())
      .def("rollback_count", &Master::RollBackCount)
      .def("detected", [](Master& m) { return m.GetCheckThread()->Detected(); });

  // --- checkpoint / data ---------------------------------------------------------------
  m.def("dump_config_data", &DumpConfigData);
  m.def("load_config_data", &LoadConfigData);
  m.def("check_fault_tolerance", &CheckFaultTolerance, py::arg("phase"), py::arg("detail") = "");
  m.def(
      "load_libsvm",
      [](const std::string& path, int shard, int num_shards, int threads, bool one_based, const std::string& assigner,
         const std::string& host, uint64_t block_size, int job_id) {
        std::vector<SVMItem> items;
        {
          py::gil_scoped_release rel;
          LoadOptions opt;
          opt.rank = shard;
          opt.num_ranks = num_shards;
          opt.num_threads = threads;
          opt.assigner = assigner;
          opt.host = host;
          opt.block_size = block_size;
          opt.job_id = job_id;
          items = LoadLibsvmFile(path, opt, one_based);
        }
        // CSR arrays: rowptr, cols, vals, labels
        std::vector<int64_t> rowptr{0}, cols;
        std::vector<double> vals, labels;
        for (auto& it : items) {
          for (auto& f : it.x) {
            cols.push_back(f.first);
            vals.push_back(f.second);
          }
          rowptr.push_back((int64_t)cols.size());
          labels.push_back(it.y);
        }
        return py::make_tuple(py::array_t<int64_t>(rowptr.size(), rowptr.data()),
                              py::array_t<int64_t>(cols.size(), cols.data()),
                              py::array_t<double>(vals.size(), vals.data()),
                              py::array_t<double>(labels.size(), labels.data()));
      },
      py::arg("path"), py::arg("shard") = 0, py::arg("num_shards") = 1, py::arg("threads") = 4,
      py::arg("one_based") = true, py::arg("assigner") = "", py::arg("host") = "", py::arg("block_size") = 0,
      py::arg("job_id") = 0);

  // --- file systems (general_fstream: local / webhdfs:// / hdfs://) and block assignment ----
  // every call that may wait on a remote file system releases the GIL (a WebHDFS peer in the
  // same process -- the tests' stand-in -- needs it to answer)
  m.def("fs_list", [](const std::string& url) {
    std::vector<FileStat> files;
    {
      py::gil_scoped_release rel;
      files = ListInputs(url);
    }
    std::vector<py::tuple> out;
    for (auto& f : files) out.push_back(py::make_tuple(f.url, f.size, f.block_size));
    return out;
  });
  m.def("fs_locations", [](const std::string& url) {
    std::vector<BlockLocation> locs;
    {
      py::gil_scoped_release rel;
      FileStat f = FileSystem::For(url).Stat(url);
      locs = FileSystem::For(url).Locations(f);
    }
    std::vector<py::tuple> out;
    for (auto& l : locs) out.push_back(py::make_tuple(l.offset, l.length, l.hosts));
    return out;
  });
  m.def("fs_read", [](const std::string& url) {
    std::string s;
    {
      py::gil_scoped_release rel;
      s = ReadFileToString(url);
    }
    return py::bytes(s);
  });
  m.def("fs_write", [](const std::string& url, const std::string& data) {
    py::gil_scoped_release rel;
    EnsureParentDir(url);
    WriteStringToFile(url, data);
  });
  m.def("fs_exists", [](const std::string& url) { return FileSystem::For(url).Exists(url); },
        py::call_guard<py::gil_scoped_release>());
  m.def("libhdfs3_available", []() {
    std::string why;
    const bool ok = LibHdfs3Available(&why);
    return py::make_tuple(ok, why);
  });
  m.def("remote_bytes_read", &RemoteBytesRead);
  m.def("local_host_name", &LocalHostName);
  py::class_<PSBoard>(m, "PSBoard")
      .def(py::init<const std::string&, int, int, int, double>(), py::arg("name"), py::arg("world"), py::arg("rank"),
           py::arg("tables"), py::arg("attach_timeout_s") = 30.0)
      .def("publish_sent", &PSBoard::PublishSent)
      .def("sent", &PSBoard::Sent)
      .def("min_sent", &PSBoard::MinSent)
      .def("publish_applied", &PSBoard::PublishApplied)
      .def("publish_applied_row", &PSBoard::PublishAppliedRow)
      .def("applied", &PSBoard::Applied)
      .def("min_applied", &PSBoard::MinApplied)
      .def("min_applied_from", &PSBoard::MinAppliedFrom)
      .def("owner_version", &PSBoard::OwnerVersion)
      .def("pending", &PSBoard::Pending)
      .def("wait_min_applied", &PSBoard::WaitMinApplied, py::arg("table"), py::arg("target"), py::arg("timeout_s"),
           py::call_guard<py::gil_scoped_release>())
      .def("wait_applied_from", &PSBoard::WaitAppliedFrom, py::arg("table"), py::arg("requester"), py::arg("target"),
           py::arg("timeout_s"), py::call_guard<py::gil_scoped_release>())
      .def("wait_sent_at_least", &PSBoard::WaitSentAtLeast, py::arg("table"), py::arg("rank"), py::arg("target"),
           py::arg("timeout_s"), py::call_guard<py::gil_scoped_release>())
      .def("snapshot_sent", &PSBoard::SnapshotSent)
      .def("snapshot_applied", &PSBoard::SnapshotApplied)
      .def("wake", &PSBoard::Wake)
      .def("read_lock", &PSBoard::ReadLock, py::arg("table"), py::arg("timeout_s"),
           py::call_guard<py::gil_scoped_release>())
      .def("read_unlock", &PSBoard::ReadUnlock)
      .def("write_lock", &PSBoard::WriteLock, py::arg("table"), py::arg("timeout_s"),
           py::call_guard<py::gil_scoped_release>())
      .def("write_unlock", &PSBoard::WriteUnlock)
      .def("set_abort", &PSBoard::SetAbort)
      .def_property_readonly("aborted", &PSBoard::Aborted)
      .def_property_readonly("wakeups", &PSBoard::Wakeups)
      .def_property_readonly("epoch", &PSBoard::Epoch)
      .def("unlink", &PSBoard::Unlink);
  py::class_<CpuAsyncServer>(m, "AsyncServer")
      .def(py::init<const std::string&, int, int, int, py::function>(), py::arg("board"), py::arg("world"),
           py::arg("rank"), py::arg("tables"), py::arg("apply"))
      .def("enable", [](CpuAsyncServer& s, int t) { s.server().Enable(t); })
      .def("set_coalesce", [](CpuAsyncServer& s, int t, bool on) { s.server().SetCoalesce(t, on); })
      .def("start", [](CpuAsyncServer& s) { s.server().Start(); })
      .def("stop", [](CpuAsyncServer& s) { s.server().Stop(); }, py::call_guard<py::gil_scoped_release>())
      .def("pause", [](CpuAsyncServer& s) { s.server().Pause(); }, py::call_guard<py::gil_scoped_release>())
      .def("resume", [](CpuAsyncServer& s) { s.server().Resume(); })
      .def("running", [](CpuAsyncServer& s) { return s.server().Running(); })
      .def("error", [](CpuAsyncServer& s) { return s.server().Error(); })
      .def("set_log", [](CpuAsyncServer& s, bool on) { s.server().SetLog(on); })
      .def("take_log", [](CpuAsyncServer& s) { return s.server().TakeLog(); })
      .def_property_readonly("applied", [](CpuAsyncServer& s) { return s.server().Applied(); })
      .def_property_readonly("batches", [](CpuAsyncServer& s) { return s.server().Batches(); });
  py::class_<BlockAssignerServer>(m, "BlockAssignerServer")
      .def(py::init<int>(), py::arg("port") = 0)
      .def("start", &BlockAssignerServer::Start)
      .def("stop", &BlockAssignerServer::Stop, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("port", &BlockAssignerServer::Port)
      .def("wait_done", &BlockAssignerServer::WaitDone, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("local_served", &BlockAssignerServer::LocalServed)
      .def_property_readonly("remote_served", &BlockAssignerServer::RemoteServed);

  // --- GPU shard checkpoint files (binary sidecar + reference text format) ---------------
  py::class_<AsyncShardWriter>(m, "ShardWriter")
      .def(py::init<>())
      .def(
          "submit",
          [](AsyncShardWriter& w, const std::string& path, const py::dict& meta, const py::list& arrays,
             const std::string& text_path) {
            ShardMeta mm = MetaFromDict(meta);
            std::vector<ArrayRef> aa = ArraysFromList(arrays);
            return w.Submit([path, mm, aa, text_path] {
              WriteShard(path, mm, aa);
              if (!text_path.empty() && !aa.empty()) WriteTextParams(text_path, aa[0]);
            });
          },
          py::arg("path"), py::arg("meta"), py::arg("arrays"), py::arg("text_path") = "")
      .def("wait", &AsyncShardWriter::Wait, py::call_guard<py::gil_scoped_release>())
      .def("wait_all", &AsyncShardWriter::WaitAll, py::call_guard<py::gil_scoped_release>())
      .def("take_error", &AsyncShardWriter::TakeError);
  py::class_<ShardFileWriter>(m, "ShardFileWriter")
      .def(py::init([](const std::string& path, const py::dict& meta, const py::list& arrays) {
             std::vector<ArrayDesc> desc;
             for (auto item : arrays) {
               auto t = item.cast<py::tuple>();
               ArrayDesc d;
               d.name = t[0].cast<std::string>();
               d.dtype = ParseDType(t[1].cast<std::string>());
               d.rows = t[2].cast<uint64_t>();
               d.cols = t[3].cast<uint64_t>();
               desc.push_back(d);
             }
             return new ShardFileWriter(path, MetaFromDict(meta), desc);
           }),
           py::arg("path"), py::arg("meta"), py::arg("arrays"))
      .def(
          "write_rows",
          [](ShardFileWriter& w, int array, uint64_t row0, uintptr_t src, uint64_t nrows) {
            py::gil_scoped_release rel;
            w.WriteRows(array, row0, reinterpret_cast<const void*>(src), nrows);
          },
          py::arg("array"), py::arg("row0"), py::arg("src"), py::arg("nrows"))
      .def("close", &ShardFileWriter::Close, py::call_guard<py::gil_scoped_release>());
  m.def(
      "read_shard_header",
      [](const std::string& path) {
        ShardHeader h;
        {
          py::gil_scoped_release rel;
          h = ReadShardHeader(path);
        }
        py::dict meta;
        meta["global_rows"] = h.meta.global_rows;
        meta["base"] = h.meta.base;
        meta["rows"] = h.meta.rows;
        meta["cols"] = h.meta.cols;
        meta["clock"] = h.meta.clock;
        meta["table_id"] = h.meta.table_id;
        meta["rank"] = h.meta.rank;
        meta["world"] = h.meta.world;
        meta["kind"] = h.meta.kind;
        py::list arrays;
        for (const auto& a : h.arrays) arrays.append(py::make_tuple(a.name, DTypeName(a.dtype), a.rows,
                                                                    a.cols, a.offset));
        return py::make_tuple(meta, arrays);
      },
      py::arg("path"));
  m.def(
      "read_rows",
      [](const std::string& path, uint64_t offset, uint64_t row_bytes, uint64_t row0, uint64_t nrows, uintptr_t dst) {
        py::gil_scoped_release rel;
        ReadRows(path, offset, row_bytes, row0, nrows, reinterpret_cast<void*>(dst));
      },
      py::arg("path"), py::arg("offset"), py::arg("row_bytes"), py::arg("row0"), py::arg("nrows"), py::arg("dst"));
  m.def(
      "write_text_params",
      [](const std::string& path, uintptr_t data, const std::string& dtype, uint64_t rows, uint64_t cols) {
        ArrayRef a;
        a.name = "params";
        a.data = reinterpret_cast<const void*>(data);
        a.dtype = ParseDType(dtype);
        a.rows = rows;
        a.cols = cols;
        py::gil_scoped_release rel;
        WriteTextParams(path, a);
      },
      py::arg("path"), py::arg("data"), py::arg("dtype"), py::arg("rows"), py::arg("cols"));
  py::class_<TextParamsWriter>(m, "TextParamsWriter")
      .def(py::init<const std::string&>(), py::call_guard<py::gil_scoped_release>())
      .def(
          "append",
          [](TextParamsWriter& w, uintptr_t data, const std::string& dtype, uint64_t rows, uint64_t cols) {
            ArrayRef a;
            a.name = "params";
            a.data = reinterpret_cast<const void*>(data);
            a.dtype = ParseDType(dtype);
            a.rows = rows;
            a.cols = cols;
            py::gil_scoped_release rel;
            w.Append(a);
          },
          py::arg("data"), py::arg("dtype"), py::arg("rows"), py::arg("cols"))
      .def("close", &TextParamsWriter::Close, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("elements", &TextParamsWriter::Elements);
  m.def("shard_bytes_read", &ShardBytesRead);
  m.def("reset_shard_bytes_read", &ResetShardBytesRead);
  m.def(
      "read_shard",
      [](const std::string& path) {
        LoadedShard s;
        {
          py::gil_scoped_release rel;
          s = ReadShard(path);
        }
        py::dict meta;
        meta["global_rows"] = s.meta.global_rows;
        meta["base"] = s.meta.base;
        meta["rows"] = s.meta.rows;
        meta["cols"] = s.meta.cols;
        meta["clock"] = s.meta.clock;
        meta["table_id"] = s.meta.table_id;
        meta["rank"] = s.meta.rank;
        meta["world"] = s.meta.world;
        meta["kind"] = s.meta.kind;
        py::list arrays;
        for (auto& a : s.arrays) {
          auto* holder = new std::vector<char>(std::move(a.bytes));
          py::capsule own(holder, [](void* p) { delete static_cast<std::vector<char>*>(p); });
          py::array_t<uint8_t> buf({(py::ssize_t)holder->size()}, {(py::ssize_t)1},
                                   reinterpret_cast<uint8_t*>(holder->data()), own);
          arrays.append(py::make_tuple(a.name, DTypeName(a.dtype), a.rows, a.cols, buf));
        }
        return py::make_tuple(meta, arrays);
      },
      py::arg("path"));
  m.def(
      "read_text_params",
      [](const std::string& path, uint64_t n) {
        std::vector<double> v;
        {
          py::gil_scoped_release rel;
          v = ReadTextParams(path, n);
        }
        return py::array_t<double>(v.size(), v.data());
      },
      py::arg("path"), py::arg("n"));
}
