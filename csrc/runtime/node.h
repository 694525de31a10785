// Node description, hostfile parsing, master selection and node-list checks.
// Parity: base/node.hpp:7-22, base/node_utils.cpp:19-109. Hostfile lines are
// `id:host:port` as in config/localnodes; an optional 4th column `:gpu` pins the rank to
// a GPU index (one process per MI355X).
#pragma once

#include <string>
#include <vector>

#include "base.h"

namespace minips {

struct Node {
  uint32_t id = 0;
  std::string hostname;
  int port = 0;
  bool is_master = false;
  int gpu = -1;
  std::string DebugString() const;
  bool operator==(const Node& o) const { return id == o.id && hostname == o.hostname && port == o.port; }
};

std::vector<Node> ParseFile(const std::string& path);
// Removes node id 1 from `nodes` and returns it as the master when heartbeat_interval > 0;
// otherwise returns a Node with is_master = false (initialised, unlike the reference).
Node SelectMaster(std::vector<Node>& nodes, int heartbeat_interval);
bool CheckValidNodeIds(const std::vector<Node>& nodes);
bool CheckUniquePort(std::vector<Node>& nodes);
Node GetNodeById(const std::vector<Node>& nodes, uint32_t id);
bool CheckConsecutiveIds(const std::vector<Node>& nodes);
bool HasNode(const std::vector<Node>& nodes, uint32_t id);

}  // namespace minips
