// Typed flag registry ("Context") with the reference's flag names.
//
// Parity: base/context.{hpp,cpp}. The reference snapshots every gflag into a string map and
// silently returns ""/0/false for unknown names; here every library flag is DECLARED with a
// type and default, lookups of undeclared names throw, and apps may
// Define() more. The per-worker iteration map (context.hpp:36-53) is mutex-protected (the
// reference writes it from many threads without a lock).
#pragma once

#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "base.h"

namespace minips {

class Context {
 public:
  enum class Type { kString, kInt, kBool, kDouble };
  static Context& Get();

  // Declare a flag (idempotent when the type matches). Returns *this for chaining.
  Context& Define(const std::string& name, Type type, const std::string& default_value,
                  const std::string& help = "");
  bool Has(const std::string& name) const;

  std::string get_string(const std::string& name) const;
  int32_t get_int32(const std::string& name) const;
  int64_t get_int64(const std::string& name) const;
  bool get_bool(const std::string& name) const;
  double get_double(const std::string& name) const;

  void set(const std::string& name, const std::string& value);
  void set(const std::string& name, const char* value) { set(name, std::string(value)); }
  void set(const std::string& name, int64_t value) { set(name, std::to_string(value)); }
  void set(const std::string& name, int value) { set(name, std::to_string(value)); }
  void set(const std::string& name, bool value) { set(name, std::string(value ? "true" : "false")); }
  void set(const std::string& name, double value);

  // Parses --name=value / --name value / --noname (bool). Unknown flags throw unless
  // allow_unknown, in which case they are returned. Returns positional args.
  std::vector<std::string> ParseArgs(int argc, const char* const* argv, bool allow_unknown = false);
  std::vector<std::string> ParseArgs(const std::vector<std::string>& args, bool allow_unknown = false);
  std::map<std::string, std::string> Snapshot() const;
  std::string Help() const;
  void ResetToDefaults();

  // worker_id -> iteration (checkpoint bookkeeping).
  void SetIteration(int worker_id, int iteration);
  int GetIteration(int worker_id) const;
  std::map<int, int> GetIterationMap() const;
  void SetIterationMap(const std::map<int, int>& m);

 private:
  Context();
  struct Entry {
    Type type;
    std::string value;
    std::string default_value;
    std::string help;
  };
  const Entry& Find(const std::string& name) const;
  mutable std::mutex mu_;
  std::map<std::string, Entry> flags_;
  std::map<int, int> iteration_map_;
};

}  // namespace minips
