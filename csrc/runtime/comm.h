// Control plane: TCP mailbox + sender actor.
//
// Parity: comm/abstract_mailbox.hpp, comm/mailbox.{hpp,cpp}, comm/sender.{hpp,cpp}.
// Design differences (MI355X build):
//   * plain TCP sockets (no ZeroMQ); one listening socket per node, one outgoing
//     connection per peer; a single poll()-driven receiver thread.
//   * same-node traffic never touches a socket: Send() dispatches it in-process (the
//     reference loops it back over TCP, comm/mailbox.cpp:51-53).
//   * engine callbacks go through MailboxHooks instead of the reference's comm -> driver /
//     lib include cycle (comm/mailbox.hpp:14, mailbox.cpp:4).
//   * Meta.failed_node_id is carried on the wire.
//   * Barrier has a timeout (barrier_timeout_s flag) instead of hanging forever.
// Bulk tensor traffic of GPU tables does NOT use this plane: it goes over RCCL/xGMI
// (minips_amd/ps).
#pragma once

#include <condition_variable>
#include <map>
#include <mutex>
#include <set>

#include "base.h"
#include "ids.h"
#include "message.h"
#include "node.h"

namespace minips {

class AbstractMailbox {
 public:
  virtual ~AbstractMailbox() = default;
  virtual int Send(const Message& msg) = 0;
};

class AbstractSender {
 public:
  virtual ~AbstractSender() = default;
  virtual void Start() = 0;
  virtual void Stop() = 0;
  virtual ThreadsafeQueue<Message>* GetMessageQueue() = 0;
};

// Engine-side reactions to control flags received by the mailbox thread.
class MailboxHooks {
 public:
  virtual ~MailboxHooks() = default;
  virtual void OnForceQuit(uint32_t node_id) {}
  virtual void OnRollBack(int failed_node_id) {}
  virtual void OnCheckpoint() {}
  virtual void OnScaleRollBack(const Node& scale_node) {}
};

class Mailbox : public AbstractMailbox {
 public:
  Mailbox(const Node& node, const std::vector<Node>& nodes, AbstractIdMapper* id_mapper,
          MailboxHooks* hooks = nullptr);
  ~Mailbox() override;

  // Binds and connects to every peer (+ master / scale node when given, id >= 0 and
  // is_master / scale flags set by the caller).
  void Start(const Node* master = nullptr, const Node* scale_node = nullptr);
  void Stop(bool barrier = true);
  int Send(const Message& msg) override;
  void RegisterQueue(uint32_t queue_id, ThreadsafeQueue<Message>* queue);
  void DeregisterQueue(uint32_t queue_id);
  size_t GetQueueMapSize();
  void Barrier();
  void ForceQuit(uint32_t node_id);
  void Update(const std::vector<Node>& nodes);
  void ConnectTo(const Node& node);  // add a peer at run time (scale-out)
  void SetScaleNode(const Node& node);
  std::vector<Node> GetNodes();
  const Node& GetNode() const { return node_; }
  // Byte / message counters (observability).
  uint64_t BytesSent() const { return bytes_sent_.load(); }
  uint64_t MessagesSent() const { return msgs_sent_.load(); }

 private:
  void Receiving();
  void Dispatch(Message&& msg);
  int SendToNode(uint32_t node_id, const Message& msg);
  int ConnectWithRetry(const Node& n, double timeout_s);
  static bool IsNodeRoutedFlag(Flag f);

  Node node_;
  std::vector<Node> nodes_;
  AbstractIdMapper* id_mapper_;
  MailboxHooks* hooks_;
  bool has_master_ = false, has_scale_ = false;
  Node master_, scale_node_;

  std::mutex nodes_mu_;
  std::mutex send_mu_;
  std::map<uint32_t, int> out_fds_;  // node id -> socket
  std::map<uint32_t, Node> peers_;   // every node we may send to

  std::mutex queue_mu_;
  std::map<uint32_t, ThreadsafeQueue<Message>*> queue_map_;

  std::mutex barrier_mu_;
  std::condition_variable barrier_cond_;
  int barrier_count_ = 0;

  int listen_fd_ = -1;
  int wake_pipe_[2] = {-1, -1};
  std::thread receiver_;
  std::atomic<bool> running_{false};
  // set once the shutdown barrier has passed: remote sends are dropped instead of reconnecting
  // (a peer that already exited would otherwise stall Stop() for the whole connect timeout)
  std::atomic<bool> stopping_{false};
  std::atomic<uint64_t> bytes_sent_{0}, msgs_sent_{0};
};

class Sender : public AbstractSender {
 public:
  explicit Sender(AbstractMailbox* mailbox) : mailbox_(mailbox) {}
  void Start() override;
  void Stop() override;
  // Blocks until every message queued before the call has been handed to the mailbox. A
  // barrier goes out on the mailbox directly, so without this it can overtake a worker's last
  // Add/Clock still waiting in the queue (the peer may then pass the barrier and stop first).
  void Flush();
  ThreadsafeQueue<Message>* GetMessageQueue() override { return &send_message_queue_; }

 private:
  void Main();
  AbstractMailbox* mailbox_;
  ThreadsafeQueue<Message> send_message_queue_;
  std::thread thread_;
  std::mutex flush_mu_;
  std::condition_variable flush_cv_;
  uint64_t flush_asked_ = 0, flush_done_ = 0;
};

}  // namespace minips
