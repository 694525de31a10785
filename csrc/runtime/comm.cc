#include "comm.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>

#include "config.h"

namespace minips {

namespace {

#pragma pack(push, 1)
struct WireHeader {
  uint32_t magic;
  int32_t sender, recver, model_id, failed_node_id;
  uint8_t flag;
  uint8_t pad[3];
  uint32_t nblobs;
};
#pragma pack(pop)
constexpr uint32_t kMagic = 0x4D505331;  // "MPS1"

bool WriteAll(int fd, const void* buf, size_t n) {
  const char* p = static_cast<const char*>(buf);
  while (n > 0) {
    ssize_t w = ::send(fd, p, n, MSG_NOSIGNAL);
    if (w < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    p += w;
    n -= (size_t)w;
  }
  return true;
}

bool ReadAll(int fd, void* buf, size_t n) {
  char* p = static_cast<char*>(buf);
  while (n > 0) {
    ssize_t r = ::recv(fd, p, n, 0);
    if (r == 0) return false;
    if (r < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    p += r;
    n -= (size_t)r;
  }
  return true;
}

// Reads one framed message; false on EOF/error.
bool ReadMessage(int fd, Message* msg) {
  WireHeader h;
  if (!ReadAll(fd, &h, sizeof(h))) return false;
  if (h.magic != kMagic) return false;
  msg->meta.sender = h.sender;
  msg->meta.recver = h.recver;
  msg->meta.model_id = h.model_id;
  msg->meta.failed_node_id = h.failed_node_id;
  msg->meta.flag = static_cast<Flag>(h.flag);
  std::vector<uint64_t> sizes(h.nblobs);
  if (h.nblobs && !ReadAll(fd, sizes.data(), sizes.size() * sizeof(uint64_t))) return false;
  msg->data.clear();
  for (uint64_t s : sizes) {
    SArray<char> blob(s);
    if (s && !ReadAll(fd, blob.data(), s)) return false;
    msg->data.push_back(blob);
  }
  return true;
}

}  // namespace

Mailbox::Mailbox(const Node& node, const std::vector<Node>& nodes, AbstractIdMapper* id_mapper, MailboxHooks* hooks)
    : node_(node), nodes_(nodes), id_mapper_(id_mapper), hooks_(hooks) {
  for (auto& n : nodes_) peers_[n.id] = n;
}

Mailbox::~Mailbox() {
  if (running_) Stop(false);
}

bool Mailbox::IsNodeRoutedFlag(Flag f) {
  switch (f) {
    case Flag::kBarrier:
    case Flag::kExit:
    case Flag::kForceQuit:
    case Flag::kHeartBeat:
    case Flag::kQuitHeartBeat:
    case Flag::kRollBack:
    case Flag::kScale:
    case Flag::kScaleRollback:
      return true;
    default:
      return false;
  }
}

int Mailbox::ConnectWithRetry(const Node& n, double timeout_s) {
  auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s);
  std::string host = n.hostname == "localhost" ? "127.0.0.1" : n.hostname;
  while (true) {
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    int rc = getaddrinfo(host.c_str(), std::to_string(n.port).c_str(), &hints, &res);
    if (rc == 0 && res) {
      int fd = ::socket(res->ai_family, res->ai_socktype, res->ai_protocol);
      if (fd >= 0 && ::connect(fd, res->ai_addr, res->ai_addrlen) == 0) {
        freeaddrinfo(res);
        int one = 1;
        setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
        return fd;
      }
      if (fd >= 0) ::close(fd);
      freeaddrinfo(res);
    }
    if (stopping_) return -1;
    if (std::chrono::steady_clock::now() > deadline) {
      MINIPS_CHECK(false, "node " << node_.id << " cannot connect to " << n.DebugString());
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
}

void Mailbox::Start(const Node* master, const Node* scale_node) {
  // Bind + listen.
  listen_fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
  MINIPS_CHECK(listen_fd_ >= 0, "socket() failed");
  int one = 1;
  setsockopt(listen_fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in addr{};
  addr.sin_family = AF_INET;
  addr.sin_addr.s_addr = htonl(INADDR_ANY);
  addr.sin_port = htons((uint16_t)node_.port);
  MINIPS_CHECK(::bind(listen_fd_, (sockaddr*)&addr, sizeof(addr)) == 0,
               "node " << node_.id << " cannot bind port " << node_.port << " errno=" << errno);
  MINIPS_CHECK(::listen(listen_fd_, 256) == 0, "listen failed");
  MINIPS_CHECK(::pipe(wake_pipe_) == 0, "pipe failed");
  running_ = true;
  receiver_ = std::thread([this] { Receiving(); });

  if (master && master->is_master) {
    has_master_ = true;
    master_ = *master;
    peers_[master_.id] = master_;
  }
  if (scale_node && scale_node->port > 0) {
    has_scale_ = true;
    scale_node_ = *scale_node;
    peers_[scale_node_.id] = scale_node_;
  }
  // Outgoing connections are opened lazily on the first Send to a peer (with retry), so a
  // process never blocks at start-up on a peer that is not up yet or has died.
  MINIPS_VLOG(1, "mailbox " << node_.id << " listening on port " << node_.port);
}

void Mailbox::ConnectTo(const Node& n) {
  std::lock_guard<std::mutex> lk(send_mu_);
  peers_[n.id] = n;
  if (n.id != node_.id && !out_fds_.count(n.id)) {
    const int fd = ConnectWithRetry(n, Context::Get().get_double("barrier_timeout_s"));
    if (fd >= 0) out_fds_[n.id] = fd;
  }
}

void Mailbox::SetScaleNode(const Node& n) {
  std::lock_guard<std::mutex> lk(nodes_mu_);
  has_scale_ = true;
  scale_node_ = n;
}

void Mailbox::Stop(bool barrier) {
  if (!running_) return;
  if (barrier) Barrier();
  stopping_ = true;
  running_ = false;
  char c = 'x';
  if (wake_pipe_[1] >= 0) (void)!::write(wake_pipe_[1], &c, 1);
  if (receiver_.joinable()) receiver_.join();
  {
    std::lock_guard<std::mutex> lk(queue_mu_);
    for (auto& kv : queue_map_) {
      Message m;
      m.meta.flag = Flag::kExit;
      kv.second->Push(m);
    }
  }
  std::lock_guard<std::mutex> lk(send_mu_);
  for (auto& kv : out_fds_) ::close(kv.second);
  out_fds_.clear();
  if (listen_fd_ >= 0) ::close(listen_fd_);
  listen_fd_ = -1;
  for (int& fd : wake_pipe_) {
    if (fd >= 0) ::close(fd);
    fd = -1;
  }
}

void Mailbox::Receiving() {
  std::vector<int> conns;
  while (running_) {
    std::vector<pollfd> pfds;
    pfds.push_back({listen_fd_, POLLIN, 0});
    pfds.push_back({wake_pipe_[0], POLLIN, 0});
    for (int fd : conns) pfds.push_back({fd, POLLIN, 0});
    int rc = ::poll(pfds.data(), pfds.size(), 500);
    if (rc < 0) {
      if (errno == EINTR) continue;
      break;
    }
    if (pfds[1].revents) break;  // woken for shutdown
    if (pfds[0].revents & POLLIN) {
      int fd = ::accept(listen_fd_, nullptr, nullptr);
      if (fd >= 0) {
        int one = 1;
        setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
        conns.push_back(fd);
      }
    }
    std::vector<int> dead;
    for (size_t i = 2; i < pfds.size(); ++i) {
      if (!pfds[i].revents) continue;
      Message msg;
      if (!ReadMessage(pfds[i].fd, &msg)) {
        dead.push_back(pfds[i].fd);
        continue;
      }
      try {
        Dispatch(std::move(msg));
      } catch (const std::exception& e) {
        MINIPS_LOG(2, "mailbox " << node_.id << " dispatch error: " << e.what());
      }
    }
    for (int fd : dead) {
      ::close(fd);
      conns.erase(std::remove(conns.begin(), conns.end(), fd), conns.end());
    }
  }
  for (int fd : conns) ::close(fd);
}

void Mailbox::Dispatch(Message&& msg) {
  switch (msg.meta.flag) {
    case Flag::kBarrier: {
      {
        std::lock_guard<std::mutex> lk(barrier_mu_);
        barrier_count_ += 1;
        MINIPS_VLOG(2, "mailbox " << node_.id << " barrier msg from " << msg.meta.sender << " count "
                                  << barrier_count_);
      }
      barrier_cond_.notify_all();
      return;
    }
    case Flag::kForceQuit: {
      {
        std::lock_guard<std::mutex> lk(nodes_mu_);
        nodes_.erase(std::remove_if(nodes_.begin(), nodes_.end(),
                                    [&](const Node& n) { return (int)n.id == msg.meta.sender; }),
                     nodes_.end());
      }
      barrier_cond_.notify_all();
      if (hooks_) hooks_->OnForceQuit((uint32_t)msg.meta.sender);
      return;
    }
    case Flag::kRollBack: {
      if (hooks_) hooks_->OnRollBack(msg.meta.sender);
      return;
    }
    case Flag::kScaleRollback: {
      if (hooks_) {
        Node n;
        n.id = (uint32_t)msg.meta.sender;
        hooks_->OnScaleRollBack(n);
      }
      return;
    }
    case Flag::kCheckpoint:
      if (hooks_) hooks_->OnCheckpoint();
      break;
    default:
      break;
  }
  // Push under queue_mu_: DeregisterQueue (same lock) then guarantees no push is in flight, so a
  // queue can be destroyed right after it is deregistered (TSan-found use-after-free otherwise).
  bool delivered = false;
  {
    std::lock_guard<std::mutex> lk(queue_mu_);
    auto it = queue_map_.find((uint32_t)msg.meta.recver);
    if (it != queue_map_.end()) {
      it->second->Push(std::move(msg));
      delivered = true;
    }
  }
  if (!delivered) {
    MINIPS_LOG(1, "mailbox " << node_.id << ": no queue for recver " << msg.meta.recver << " ("
                             << FlagName(msg.meta.flag) << "), dropped");
  }
}

int Mailbox::SendToNode(uint32_t node_id, const Message& msg) {
  if (node_id == node_.id) {
    Message copy = msg;  // in-process fast path
    Dispatch(std::move(copy));
    return 0;
  }
  WireHeader h{};
  h.magic = kMagic;
  h.sender = msg.meta.sender;
  h.recver = msg.meta.recver;
  h.model_id = msg.meta.model_id;
  h.failed_node_id = msg.meta.failed_node_id;
  h.flag = static_cast<uint8_t>(msg.meta.flag);
  h.nblobs = (uint32_t)msg.data.size();
  std::vector<uint64_t> sizes;
  size_t total = sizeof(h);
  for (auto& d : msg.data) {
    sizes.push_back(d.size());
    total += d.size() + sizeof(uint64_t);
  }
  std::lock_guard<std::mutex> lk(send_mu_);
  auto it = out_fds_.find(node_id);
  if (it == out_fds_.end()) {
    if (stopping_) {
      MINIPS_VLOG(1, "mailbox " << node_.id << ": stopping, dropped " << FlagName(msg.meta.flag) << " to node "
                                << node_id);
      return -1;
    }
    auto pit = peers_.find(node_id);
    MINIPS_CHECK(pit != peers_.end(), "node " << node_.id << ": unknown destination node " << node_id);
    const int nfd = ConnectWithRetry(pit->second, Context::Get().get_double("barrier_timeout_s"));
    if (nfd < 0) return -1;
    out_fds_[node_id] = nfd;
    it = out_fds_.find(node_id);
  }
  int fd = it->second;
  bool ok = WriteAll(fd, &h, sizeof(h));
  if (ok && !sizes.empty()) ok = WriteAll(fd, sizes.data(), sizes.size() * sizeof(uint64_t));
  for (size_t i = 0; ok && i < msg.data.size(); ++i)
    if (msg.data[i].size()) ok = WriteAll(fd, msg.data[i].data(), msg.data[i].size());
  if (!ok) {
    MINIPS_LOG(1, "mailbox " << node_.id << ": send of " << FlagName(msg.meta.flag) << " (" << msg.meta.sender
                             << " -> " << msg.meta.recver << ") to node " << node_id << " failed");
    ::close(fd);
    out_fds_.erase(node_id);
    return -1;
  }
  bytes_sent_ += total;
  msgs_sent_ += 1;
  return (int)total;
}

int Mailbox::Send(const Message& msg) {
  uint32_t node_id = IsNodeRoutedFlag(msg.meta.flag) ? (uint32_t)msg.meta.recver
                                                     : id_mapper_->GetNodeIdForThread((uint32_t)msg.meta.recver);
  return SendToNode(node_id, msg);
}

void Mailbox::RegisterQueue(uint32_t queue_id, ThreadsafeQueue<Message>* queue) {
  std::lock_guard<std::mutex> lk(queue_mu_);
  MINIPS_CHECK(!queue_map_.count(queue_id), "queue " << queue_id << " already registered");
  queue_map_[queue_id] = queue;
}

void Mailbox::DeregisterQueue(uint32_t queue_id) {
  std::lock_guard<std::mutex> lk(queue_mu_);
  queue_map_.erase(queue_id);
}

size_t Mailbox::GetQueueMapSize() {
  std::lock_guard<std::mutex> lk(queue_mu_);
  return queue_map_.size();
}

std::vector<Node> Mailbox::GetNodes() {
  std::lock_guard<std::mutex> lk(nodes_mu_);
  return nodes_;
}

void Mailbox::Barrier() {
  std::vector<Node> targets = GetNodes();
  {
    std::lock_guard<std::mutex> lk(nodes_mu_);
    if (has_scale_ && !HasNode(targets, scale_node_.id)) targets.push_back(scale_node_);
  }
  for (auto& n : targets) {
    Message m;
    m.meta.sender = (int32_t)node_.id;
    m.meta.recver = (int32_t)n.id;
    m.meta.flag = Flag::kBarrier;
    Send(m);
  }
  double timeout = Context::Get().get_double("barrier_timeout_s");
  std::unique_lock<std::mutex> lk(barrier_mu_);
  auto target = [&] {
    std::lock_guard<std::mutex> nl(nodes_mu_);
    return (int)nodes_.size() + ((has_scale_ && !HasNode(nodes_, scale_node_.id)) ? 1 : 0);
  };
  bool ok = CondWaitFor(barrier_cond_, lk, timeout, [&] { return barrier_count_ >= target(); });
  MINIPS_CHECK(ok, "node " << node_.id << " barrier timed out (" << barrier_count_ << "/" << target() << ")");
  MINIPS_VLOG(2, "mailbox " << node_.id << " barrier passed (" << barrier_count_ << "/" << target() << ")");
  barrier_count_ -= target();
}

void Mailbox::ForceQuit(uint32_t node_id) {
  for (auto& n : GetNodes()) {
    Message m;
    m.meta.sender = (int32_t)node_id;
    m.meta.recver = (int32_t)n.id;
    m.meta.flag = Flag::kForceQuit;
    Send(m);
  }
}

void Mailbox::Update(const std::vector<Node>& nodes) {
  std::lock_guard<std::mutex> lk(nodes_mu_);
  nodes_ = nodes;
}

void Sender::Start() {
  thread_ = std::thread([this] { Main(); });
}

void Sender::Stop() {
  Message m;
  m.meta.flag = Flag::kExit;
  send_message_queue_.Push(m);
  if (thread_.joinable()) thread_.join();
}

// Flush marker: a kExit addressed to recver -2 (never a real thread id).
constexpr int32_t kFlushMarker = -2;

void Sender::Flush() {
  if (!thread_.joinable()) return;
  uint64_t ticket;
  {
    std::lock_guard<std::mutex> lk(flush_mu_);
    ticket = ++flush_asked_;
  }
  Message m;
  m.meta.flag = Flag::kExit;
  m.meta.recver = kFlushMarker;
  send_message_queue_.Push(m);
  std::unique_lock<std::mutex> lk(flush_mu_);
  flush_cv_.wait(lk, [&] { return flush_done_ >= ticket; });
}

void Sender::Main() {
  while (true) {
    Message msg;
    send_message_queue_.WaitAndPop(&msg);
    if (msg.meta.flag == Flag::kExit && msg.meta.recver == kFlushMarker) {
      {
        std::lock_guard<std::mutex> lk(flush_mu_);
        ++flush_done_;
      }
      flush_cv_.notify_all();
      continue;
    }
    if (msg.meta.flag == Flag::kExit && msg.meta.recver < 0) break;
    try {
      mailbox_->Send(msg);
    } catch (const std::exception& e) {
      MINIPS_LOG(2, "sender: " << e.what());
    }
  }
}

}  // namespace minips
