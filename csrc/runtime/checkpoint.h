// Worker-side checkpoint I/O, libsvm parsing, data loading and batch sampling.
//
// Parity:
//   DumpSVMData / LoadSVMData   -> lib/svm_dumper.hpp:25-45,128-173 (`label idx:val ...`,
//                                  0-based idx in the dump; reload parses 0-based -- the
//                                  reference re-subtracted 1: fixed)
//   DumpConfigData / LoadConfigData -> lib/svm_dumper.hpp:51-93 (`wid:iter ...`)
//   DumpScaleFile / LoadScaleFile   -> lib/svm_dumper.hpp:95-126 (`id:host:port`)
//   ParseLibsvm                 -> lib/parser.hpp:17-47 (1-based file idx -> 0-based)
//   LoadLibsvmFile              -> lib/abstract_data_loader.hpp + io/line_input_format.hpp
//                                  (local FS, multi-threaded chunked parse; node r of n
//                                  takes byte-range shard r, the HDFS-block analogue)
//   BatchDataSampler            -> lib/batch_data_sampler.cpp:23-86
//   CheckFaultTolerance         -> base/utils.hpp:24-53 ("[Fault Tolerance][PhaseN][ts]")
#pragma once

#include <map>
#include <random>
#include <string>
#include <vector>

#include "base.h"
#include "io.h"
#include "node.h"

namespace minips {

struct SVMItem {
  std::vector<std::pair<int64_t, double>> x;  // (0-based feature idx, value)
  double y = 0;
};

void EnsureParentDir(const std::string& path);

void DumpSVMData(const std::string& path, const std::vector<SVMItem>& data);
std::vector<SVMItem> LoadSVMData(const std::string& path);  // 0-based idx file
void DumpConfigData(const std::string& path, const std::map<int, int>& iteration_map);
std::map<int, int> LoadConfigData(const std::string& path);
void DumpScaleFile(const std::string& path, const Node& node);
Node LoadScaleFile(const std::string& path);

// `one_based` = true for raw libsvm files (subtract 1), false for the 0-based dumps.
bool ParseLibsvm(const char* line, size_t len, SVMItem* out, bool one_based = true);
// Reads shard `shard` of `num_shards` (split by byte range on line boundaries) with
// `num_threads` parser threads.
std::vector<SVMItem> LoadLibsvmFile(const std::string& path, int shard = 0, int num_shards = 1,
                                    int num_threads = 4, bool one_based = true);
// Same, with the full loader options (block assigner service, locality host, block size).
std::vector<SVMItem> LoadLibsvmFile(const std::string& path, const LoadOptions& opt, bool one_based = true);

class BatchDataSampler {
 public:
  BatchDataSampler(const std::vector<SVMItem>* data, int batch_size, uint64_t seed = 0);
  void RandomStartPoint();
  // Returns the sorted unique feature keys of the next batch (std::set semantics).
  std::vector<Key> PrepareNextBatch();
  const std::vector<const SVMItem*>& GetDataPtrs() const { return batch_ptrs_; }
  int BatchSize() const { return batch_size_; }

 private:
  const std::vector<SVMItem>* data_;
  int batch_size_;
  size_t current_ = 0;
  std::mt19937_64 rng_;
  std::vector<const SVMItem*> batch_ptrs_;
};

// Fault-tolerance phase log line (phases 2..5: detect, restart, recover, others recovered).
void CheckFaultTolerance(int phase, const std::string& detail = "");

}  // namespace minips
