#include "fs.h"

#include <dirent.h>
#include <dlfcn.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>

namespace minips {

namespace {

std::atomic<uint64_t> g_remote_bytes{0};

// ------------------------------------------------------------------------------------------
// Minimal JSON reader: enough for WebHDFS replies (objects, arrays, strings, numbers, bools).
// ------------------------------------------------------------------------------------------
struct Json {
  enum Kind { kNull, kBool, kNum, kStr, kArr, kObj } kind = kNull;
  double num = 0;
  bool b = false;
  std::string str;
  std::vector<Json> arr;
  std::vector<std::pair<std::string, Json>> obj;

  const Json* Get(const std::string& k) const {
    for (auto& kv : obj)
      if (kv.first == k) return &kv.second;
    return nullptr;
  }
  const Json& At(const std::string& k) const {
    const Json* j = Get(k);
    MINIPS_CHECK(j != nullptr, "JSON reply has no field '" << k << "'");
    return *j;
  }
};

class JsonParser {
 public:
  explicit JsonParser(const std::string& s) : s_(s) {}
  Json Parse() {
    Json j = Value();
    Ws();
    MINIPS_CHECK(i_ == s_.size(), "trailing bytes in JSON at " << i_);
    return j;
  }

 private:
  void Ws() {
    while (i_ < s_.size() && (s_[i_] == ' ' || s_[i_] == '\n' || s_[i_] == '\r' || s_[i_] == '\t')) ++i_;
  }
  char Peek() {
    Ws();
    MINIPS_CHECK(i_ < s_.size(), "truncated JSON");
    return s_[i_];
  }
  void Expect(char c) {
    MINIPS_CHECK(Peek() == c, "JSON: expected '" << c << "' at " << i_);
    ++i_;
  }
  std::string Str() {
    Expect('"');
    std::string out;
    while (i_ < s_.size() && s_[i_] != '"') {
      char c = s_[i_++];
      if (c == '\\') {
        MINIPS_CHECK(i_ < s_.size(), "truncated JSON escape");
        char e = s_[i_++];
        switch (e) {
          case 'n': out += '\n'; break;
          case 't': out += '\t'; break;
          case 'r': out += '\r'; break;
          case 'b': out += '\b'; break;
          case 'f': out += '\f'; break;
          case 'u': {  // BMP code point -> UTF-8 (HDFS names are UTF-8; surrogates kept as-is)
            MINIPS_CHECK(i_ + 4 <= s_.size(), "truncated \\u escape");
            unsigned cp = (unsigned)std::stoul(s_.substr(i_, 4), nullptr, 16);
            i_ += 4;
            if (cp < 0x80) {
              out += (char)cp;
            } else if (cp < 0x800) {
              out += (char)(0xC0 | (cp >> 6));
              out += (char)(0x80 | (cp & 0x3F));
            } else {
              out += (char)(0xE0 | (cp >> 12));
              out += (char)(0x80 | ((cp >> 6) & 0x3F));
              out += (char)(0x80 | (cp & 0x3F));
            }
            break;
          }
          default: out += e;
        }
      } else {
        out += c;
      }
    }
    Expect('"');
    return out;
  }
  Json Value() {
    Json j;
    char c = Peek();
    if (c == '{') {
      j.kind = Json::kObj;
      ++i_;
      if (Peek() == '}') {
        ++i_;
        return j;
      }
      for (;;) {
        std::string k = Str();
        Expect(':');
        j.obj.emplace_back(std::move(k), Value());
        if (Peek() == ',') {
          ++i_;
          continue;
        }
        Expect('}');
        return j;
      }
    }
    if (c == '[') {
      j.kind = Json::kArr;
      ++i_;
      if (Peek() == ']') {
        ++i_;
        return j;
      }
      for (;;) {
        j.arr.push_back(Value());
        if (Peek() == ',') {
          ++i_;
          continue;
        }
        Expect(']');
        return j;
      }
    }
    if (c == '"') {
      j.kind = Json::kStr;
      j.str = Str();
      return j;
    }
    if (s_.compare(i_, 4, "true") == 0 || s_.compare(i_, 5, "false") == 0) {
      j.kind = Json::kBool;
      j.b = s_[i_] == 't';
      i_ += j.b ? 4 : 5;
      return j;
    }
    if (s_.compare(i_, 4, "null") == 0) {
      i_ += 4;
      return j;
    }
    const char* p = s_.c_str() + i_;
    char* q = nullptr;
    j.kind = Json::kNum;
    j.num = std::strtod(p, &q);
    MINIPS_CHECK(q != p, "JSON: bad value at " << i_);
    i_ += (size_t)(q - p);
    return j;
  }
  const std::string& s_;
  size_t i_ = 0;
};

// ------------------------------------------------------------------------------------------
// HTTP/1.1 client over a plain TCP socket (one request per connection).
// ------------------------------------------------------------------------------------------
struct HttpResponse {
  int status = 0;
  std::map<std::string, std::string> headers;  // lower-case names
  std::string body;
};

int TcpConnect(const std::string& host_in, int port) {
  const std::string host = host_in == "localhost" ? "127.0.0.1" : host_in;
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  int rc = getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res);
  MINIPS_CHECK(rc == 0 && res, "cannot resolve " << host << ":" << port);
  int fd = ::socket(res->ai_family, res->ai_socktype, res->ai_protocol);
  const bool ok = fd >= 0 && ::connect(fd, res->ai_addr, res->ai_addrlen) == 0;
  freeaddrinfo(res);
  if (!ok) {
    if (fd >= 0) ::close(fd);
    MINIPS_CHECK(false, "cannot connect to " << host << ":" << port << " errno=" << errno);
  }
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  timeval tv{120, 0};  // a dead datanode fails the read / write instead of hanging the loader
  setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
  setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
  return fd;
}

void SendAll(int fd, const char* p, size_t n) {
  while (n > 0) {
    ssize_t w = ::send(fd, p, n, MSG_NOSIGNAL);
    if (w < 0 && errno == EINTR) continue;
    MINIPS_CHECK(w > 0, "HTTP send failed errno=" << errno);
    p += w;
    n -= (size_t)w;
  }
}

class SocketReader {
 public:
  explicit SocketReader(int fd) : fd_(fd) {}
  // false at EOF
  bool Fill() {
    char tmp[1 << 16];
    for (;;) {
      ssize_t r = ::recv(fd_, tmp, sizeof(tmp), 0);
      if (r < 0 && errno == EINTR) continue;
      MINIPS_CHECK(r >= 0, "HTTP recv failed errno=" << errno);
      if (r == 0) return false;
      buf_.append(tmp, (size_t)r);
      return true;
    }
  }
  std::string Line() {
    for (;;) {
      size_t p = buf_.find("\r\n", pos_);
      if (p != std::string::npos) {
        std::string l = buf_.substr(pos_, p - pos_);
        pos_ = p + 2;
        return l;
      }
      MINIPS_CHECK(Fill(), "HTTP: connection closed inside a header");
    }
  }
  void Take(size_t n, std::string* out) {
    while (buf_.size() - pos_ < n) MINIPS_CHECK(Fill(), "HTTP: connection closed inside a body");
    out->append(buf_, pos_, n);
    pos_ += n;
    Compact();
  }
  void Rest(std::string* out) {
    while (Fill()) {
    }
    out->append(buf_, pos_, std::string::npos);
    pos_ = buf_.size();
  }

 private:
  void Compact() {
    if (pos_ > (1 << 20)) {
      buf_.erase(0, pos_);
      pos_ = 0;
    }
  }
  int fd_;
  std::string buf_;
  size_t pos_ = 0;
};

HttpResponse HttpRequest(const std::string& method, const std::string& host, int port, const std::string& target,
                         const char* body = nullptr, size_t body_len = 0) {
  int fd = TcpConnect(host, port);
  struct Closer {
    int fd;
    ~Closer() { ::close(fd); }
  } closer{fd};
  std::string req = method + " " + target + " HTTP/1.1\r\nHost: " + host + ":" + std::to_string(port) +
                    "\r\nConnection: close\r\nAccept: */*\r\n";
  if (body || method == "PUT" || method == "POST") {
    req += "Content-Type: application/octet-stream\r\nContent-Length: " + std::to_string(body_len) + "\r\n";
  }
  req += "\r\n";
  SendAll(fd, req.data(), req.size());
  if (body_len) SendAll(fd, body, body_len);
  SocketReader rd(fd);
  HttpResponse r;
  const std::string status = rd.Line();  // HTTP/1.1 200 OK
  MINIPS_CHECK(status.compare(0, 5, "HTTP/") == 0, "not an HTTP reply: " << status);
  r.status = std::atoi(status.c_str() + status.find(' ') + 1);
  for (;;) {
    std::string l = rd.Line();
    if (l.empty()) break;
    size_t c = l.find(':');
    if (c == std::string::npos) continue;
    std::string k = l.substr(0, c), v = l.substr(c + 1);
    std::transform(k.begin(), k.end(), k.begin(), ::tolower);
    v.erase(0, v.find_first_not_of(' '));
    while (!v.empty() && (v.back() == ' ' || v.back() == '\r')) v.pop_back();
    r.headers[k] = v;
  }
  if (method == "HEAD" || r.status == 204 || r.status == 304) return r;
  auto te = r.headers.find("transfer-encoding");
  auto cl = r.headers.find("content-length");
  if (te != r.headers.end() && te->second.find("chunked") != std::string::npos) {
    for (;;) {
      const size_t n = std::strtoull(rd.Line().c_str(), nullptr, 16);
      if (n == 0) break;
      rd.Take(n, &r.body);
      rd.Line();
    }
  } else if (cl != r.headers.end()) {
    rd.Take(std::strtoull(cl->second.c_str(), nullptr, 10), &r.body);
  } else {
    rd.Rest(&r.body);
  }
  return r;
}

std::string PercentEncode(const std::string& s) {
  static const char* hex = "0123456789ABCDEF";
  std::string out;
  for (unsigned char c : s) {
    if (std::isalnum(c) || c == '/' || c == '-' || c == '_' || c == '.' || c == '~') {
      out += (char)c;
    } else {
      out += '%';
      out += hex[c >> 4];
      out += hex[c & 15];
    }
  }
  return out;
}

std::string JoinPath(const std::string& dir, const std::string& name) {
  if (name.empty()) return dir;
  return dir + (!dir.empty() && dir.back() == '/' ? "" : "/") + name;
}

// ------------------------------------------------------------------------------------------
// Local POSIX file system.
// ------------------------------------------------------------------------------------------
std::string LocalPath(const std::string& url) {
  const Url u = ParseUrl(url);
  return u.path;
}

class LocalFile : public RandomAccessFile {
 public:
  explicit LocalFile(const std::string& path) {
    fd_ = ::open(path.c_str(), O_RDONLY);
    MINIPS_CHECK(fd_ >= 0, "cannot open " << path);
    struct stat st;
    MINIPS_CHECK(::fstat(fd_, &st) == 0, "cannot stat " << path);
    size_ = (uint64_t)st.st_size;
  }
  ~LocalFile() override { ::close(fd_); }
  uint64_t Size() const override { return size_; }
  size_t ReadAt(uint64_t off, char* buf, size_t n) override {
    size_t got = 0;
    while (got < n) {
      ssize_t r = ::pread(fd_, buf + got, n - got, (off_t)(off + got));
      if (r < 0 && errno == EINTR) continue;
      MINIPS_CHECK(r >= 0, "pread failed errno=" << errno);
      if (r == 0) break;
      got += (size_t)r;
    }
    return got;
  }

 private:
  int fd_ = -1;
  uint64_t size_ = 0;
};

class LocalWritable : public WritableFile {
 public:
  explicit LocalWritable(const std::string& path) : path_(path) {
    f_ = std::fopen(path.c_str(), "wb");
    MINIPS_CHECK(f_ != nullptr, "cannot write " << path << " errno=" << errno);
  }
  ~LocalWritable() override {
    if (f_) std::fclose(f_);
  }
  void Append(const char* d, size_t n) override {
    MINIPS_CHECK(f_ && std::fwrite(d, 1, n, f_) == n, "short write to " << path_);
  }
  void Close() override {
    if (!f_) return;
    const bool ok = std::fflush(f_) == 0;
    std::fclose(f_);
    f_ = nullptr;
    MINIPS_CHECK(ok, "flush failed for " << path_);
  }

 private:
  std::string path_;
  FILE* f_ = nullptr;
};

class LocalFs : public FileSystem {
 public:
  std::string Name() const override { return "local"; }
  FileStat Stat(const std::string& url) override {
    struct stat st;
    const std::string p = LocalPath(url);
    MINIPS_CHECK(::stat(p.c_str(), &st) == 0, "no such file " << url);
    FileStat f;
    f.url = url;
    f.size = S_ISDIR(st.st_mode) ? 0 : (uint64_t)st.st_size;
    f.is_dir = S_ISDIR(st.st_mode);
    return f;
  }
  bool Exists(const std::string& url) override {
    struct stat st;
    return ::stat(LocalPath(url).c_str(), &st) == 0;
  }
  std::vector<FileStat> List(const std::string& url) override {
    FileStat top = Stat(url);
    if (!top.is_dir) return {top};
    std::vector<std::string> names;
    DIR* d = ::opendir(LocalPath(url).c_str());
    MINIPS_CHECK(d != nullptr, "cannot open directory " << url);
    while (dirent* e = ::readdir(d)) {
      std::string n = e->d_name;
      if (n != "." && n != "..") names.push_back(n);
    }
    ::closedir(d);
    std::sort(names.begin(), names.end());
    std::vector<FileStat> out;
    for (auto& n : names) {
      FileStat f = Stat(JoinPath(url, n));
      if (!f.is_dir) out.push_back(f);
    }
    return out;
  }
  std::vector<BlockLocation> Locations(const FileStat& f) override {
    // every byte of a local (or NFS-mounted) file is "on" this host: one location entry
    return {BlockLocation{0, f.size, {LocalHostName()}}};
  }
  std::unique_ptr<RandomAccessFile> OpenRead(const std::string& url) override {
    return std::unique_ptr<RandomAccessFile>(new LocalFile(LocalPath(url)));
  }
  std::unique_ptr<WritableFile> OpenWrite(const std::string& url) override {
    return std::unique_ptr<WritableFile>(new LocalWritable(LocalPath(url)));
  }
  void MakeDirs(const std::string& url) override {
    std::string p = LocalPath(url), cur;
    for (size_t i = 0; i <= p.size(); ++i) {
      if (i == p.size() || (p[i] == '/' && i > 0)) {
        cur = p.substr(0, i);
        if (::mkdir(cur.c_str(), 0755) != 0 && errno != EEXIST) MINIPS_CHECK(false, "mkdir " << cur);
      }
    }
  }
  void Rename(const std::string& a, const std::string& b) override {
    MINIPS_CHECK(::rename(LocalPath(a).c_str(), LocalPath(b).c_str()) == 0, "rename " << a << " -> " << b);
  }
  void Remove(const std::string& url) override { ::unlink(LocalPath(url).c_str()); }
};

// ------------------------------------------------------------------------------------------
// WebHDFS (REST) client: webhdfs://namenode:http_port/path
// ------------------------------------------------------------------------------------------
class WebHdfs : public FileSystem {
 public:
  WebHdfs(std::string host, int port) : host_(std::move(host)), port_(port) {
    if (const char* u = std::getenv("HADOOP_USER_NAME")) user_ = u;
  }
  std::string Name() const override { return "webhdfs://" + host_ + ":" + std::to_string(port_); }

  // One namenode call; redirects (307 to a datanode) are followed with the same method + body.
  HttpResponse Call(const std::string& method, const std::string& path, const std::string& op,
                    const std::string& extra = "", const char* body = nullptr, size_t len = 0) {
    std::string target = "/webhdfs/v1" + PercentEncode(path) + "?op=" + op + extra;
    if (!user_.empty()) target += "&user.name=" + user_;
    std::string host = host_;
    int port = port_;
    for (int hop = 0; hop < 4; ++hop) {
      const bool to_namenode = hop == 0;
      // the namenode step of a CREATE/APPEND carries no data (it only answers with a redirect)
      const bool send_body = !to_namenode || !(op == "CREATE" || op == "APPEND");
      HttpResponse r = HttpRequest(method, host, port, target, send_body ? body : nullptr, send_body ? len : 0);
      if (r.status == 307 || r.status == 302 || r.status == 301) {
        const Url loc = ParseUrl(r.headers["location"]);
        MINIPS_CHECK(!loc.host.empty(), "WebHDFS redirect without a host: " << r.headers["location"]);
        host = loc.host;
        port = loc.port ? loc.port : 80;
        target = loc.path + (loc.query.empty() ? "" : "?" + loc.query);
        continue;
      }
      if (r.status / 100 != 2) {
        std::string msg = r.body.substr(0, 300);
        try {
          Json j = JsonParser(r.body).Parse();
          if (const Json* e = j.Get("RemoteException"))
            if (const Json* m = e->Get("message")) msg = m->str;
        } catch (const std::exception&) {
        }
        throw CheckError("WebHDFS " + op + " " + path + " on " + Name() + " failed: HTTP " +
                         std::to_string(r.status) + " " + msg);
      }
      return r;
    }
    throw CheckError("WebHDFS " + op + " " + path + ": too many redirects");
  }

  FileStat FromStatus(const std::string& url, const Json& s) {
    FileStat f;
    f.url = url;
    f.is_dir = s.At("type").str == "DIRECTORY";
    f.size = (uint64_t)s.At("length").num;
    if (const Json* bs = s.Get("blockSize")) f.block_size = (uint64_t)bs->num;
    return f;
  }
  FileStat Stat(const std::string& url) override {
    const Url u = ParseUrl(url);
    Json j = JsonParser(Call("GET", u.path, "GETFILESTATUS").body).Parse();
    return FromStatus(url, j.At("FileStatus"));
  }
  bool Exists(const std::string& url) override {
    try {
      Stat(url);
      return true;
    } catch (const CheckError& e) {
      if (std::string(e.what()).find("HTTP 404") != std::string::npos) return false;
      throw;
    }
  }
  std::vector<FileStat> List(const std::string& url) override {
    FileStat top = Stat(url);
    if (!top.is_dir) return {top};
    const Url u = ParseUrl(url);
    Json j = JsonParser(Call("GET", u.path, "LISTSTATUS").body).Parse();
    std::vector<FileStat> out;
    for (auto& s : j.At("FileStatuses").At("FileStatus").arr) {
      FileStat f = FromStatus(JoinPath(url, s.At("pathSuffix").str), s);
      if (!f.is_dir) out.push_back(f);
    }
    std::sort(out.begin(), out.end(), [](const FileStat& a, const FileStat& b) { return a.url < b.url; });
    return out;
  }
  std::vector<BlockLocation> Locations(const FileStat& f) override {
    const Url u = ParseUrl(f.url);
    std::vector<BlockLocation> out;
    const std::string range = "&offset=0&length=" + std::to_string(f.size);
    try {  // public API (Hadoop >= 3.3): {"BlockLocations":{"BlockLocation":[{offset,length,hosts}]}}
      Json j = JsonParser(Call("GET", u.path, "GETFILEBLOCKLOCATIONS", range).body).Parse();
      for (auto& b : j.At("BlockLocations").At("BlockLocation").arr) {
        BlockLocation l{(uint64_t)b.At("offset").num, (uint64_t)b.At("length").num, {}};
        for (auto& h : b.At("hosts").arr) l.hosts.push_back(h.str);
        out.push_back(std::move(l));
      }
      return out;
    } catch (const CheckError&) {
    }
    // older namenodes: {"LocatedBlocks":{"locatedBlocks":[{startOffset, block{numBytes}, locations[{hostName}]}]}}
    Json j = JsonParser(Call("GET", u.path, "GET_BLOCK_LOCATIONS", range).body).Parse();
    for (auto& b : j.At("LocatedBlocks").At("locatedBlocks").arr) {
      BlockLocation l{(uint64_t)b.At("startOffset").num, (uint64_t)b.At("block").At("numBytes").num, {}};
      for (auto& h : b.At("locations").arr) l.hosts.push_back(h.At("hostName").str);
      out.push_back(std::move(l));
    }
    return out;
  }

  class Reader : public RandomAccessFile {
   public:
    Reader(WebHdfs* fs, std::string path, uint64_t size) : fs_(fs), path_(std::move(path)), size_(size) {}
    uint64_t Size() const override { return size_; }
    size_t ReadAt(uint64_t off, char* buf, size_t n) override {
      if (off >= size_) return 0;
      n = (size_t)std::min<uint64_t>(n, size_ - off);
      if (n == 0) return 0;
      const std::string range = "&offset=" + std::to_string(off) + "&length=" + std::to_string(n);
      HttpResponse r = fs_->Call("GET", path_, "OPEN", range);
      const size_t got = std::min(n, r.body.size());
      std::memcpy(buf, r.body.data(), got);
      g_remote_bytes += got;
      return got;
    }

   private:
    WebHdfs* fs_;
    std::string path_;
    uint64_t size_;
  };
  std::unique_ptr<RandomAccessFile> OpenRead(const std::string& url) override {
    FileStat f = Stat(url);
    MINIPS_CHECK(!f.is_dir, url << " is a directory");
    return std::unique_ptr<RandomAccessFile>(new Reader(this, ParseUrl(url).path, f.size));
  }

  // Buffered writer: CREATE with the first buffer, APPEND for every later one (bounded memory).
  class Writer : public WritableFile {
   public:
    Writer(WebHdfs* fs, std::string path) : fs_(fs), path_(std::move(path)) {}
    ~Writer() override {
      try {
        if (!closed_) Close();
      } catch (const std::exception&) {
      }
    }
    void Append(const char* d, size_t n) override {
      buf_.append(d, n);
      if (buf_.size() >= kFlush) Flush();
    }
    void Close() override {
      if (closed_) return;
      if (!created_ || !buf_.empty()) Flush();
      closed_ = true;
    }

   private:
    static constexpr size_t kFlush = 32 << 20;
    void Flush() {
      if (!created_) {
        fs_->Call("PUT", path_, "CREATE", "&overwrite=true", buf_.data(), buf_.size());
        created_ = true;
      } else {
        fs_->Call("POST", path_, "APPEND", "", buf_.data(), buf_.size());
      }
      buf_.clear();
    }
    WebHdfs* fs_;
    std::string path_, buf_;
    bool created_ = false, closed_ = false;
  };
  std::unique_ptr<WritableFile> OpenWrite(const std::string& url) override {
    return std::unique_ptr<WritableFile>(new Writer(this, ParseUrl(url).path));
  }
  void MakeDirs(const std::string& url) override { Call("PUT", ParseUrl(url).path, "MKDIRS"); }
  void Rename(const std::string& a, const std::string& b) override {
    Call("PUT", ParseUrl(a).path, "RENAME", "&destination=" + PercentEncode(ParseUrl(b).path));
  }
  void Remove(const std::string& url) override { Call("DELETE", ParseUrl(url).path, "DELETE", "&recursive=true"); }

 private:
  std::string host_;
  int port_;
  std::string user_;
};

// ------------------------------------------------------------------------------------------
// libhdfs3 (native HDFS RPC), resolved with dlopen at first use.
// ------------------------------------------------------------------------------------------
struct HdfsFileInfoAbi {  // hdfs.h hdfsFileInfo
  int mKind;              // 'F' file, 'D' directory
  char* mName;
  long mLastMod;
  int64_t mSize;
  short mReplication;
  int64_t mBlockSize;
  char* mOwner;
  char* mGroup;
  short mPermissions;
  long mLastAccess;
};

struct LibHdfs3 {
  void* h = nullptr;
  std::string error;
  void* (*connect)(const char*, uint16_t) = nullptr;
  int (*disconnect)(void*) = nullptr;
  void* (*open)(void*, const char*, int, int, short, int32_t) = nullptr;
  int (*close)(void*, void*) = nullptr;
  int32_t (*pread)(void*, void*, int64_t, void*, int32_t) = nullptr;
  int32_t (*write)(void*, void*, const void*, int32_t) = nullptr;
  HdfsFileInfoAbi* (*path_info)(void*, const char*) = nullptr;
  HdfsFileInfoAbi* (*list)(void*, const char*, int*) = nullptr;
  void (*free_info)(HdfsFileInfoAbi*, int) = nullptr;
  char*** (*hosts)(void*, const char*, int64_t, int64_t) = nullptr;
  void (*free_hosts)(char***) = nullptr;
  int (*exists)(void*, const char*) = nullptr;
  int (*mkdir)(void*, const char*) = nullptr;
  int (*rename)(void*, const char*, const char*) = nullptr;
  int (*del)(void*, const char*, int) = nullptr;

  static LibHdfs3& Get() {
    static LibHdfs3 lib;
    static std::once_flag once;
    std::call_once(once, [] { lib.Load(); });
    return lib;
  }
  template <class F>
  void Sym(F* f, const char* name) {
    *f = reinterpret_cast<F>(::dlsym(h, name));
    if (!*f && error.empty()) error = std::string("libhdfs3 lacks ") + name;
  }
  void Load() {
    const char* env = std::getenv("MINIPS_LIBHDFS3");
    for (const char* cand : {env, "libhdfs3.so", "libhdfs3.so.1"}) {
      if (cand && (h = ::dlopen(cand, RTLD_NOW | RTLD_LOCAL))) break;
    }
    if (!h) {
      error = "libhdfs3 is not installed (dlopen libhdfs3.so failed); read hdfs:// data through the namenode's "
              "REST API as webhdfs://<namenode>:<http port>/path, or set MINIPS_HDFS_HTTP_PORT";
      return;
    }
    Sym(&connect, "hdfsConnect");
    Sym(&disconnect, "hdfsDisconnect");
    Sym(&open, "hdfsOpenFile");
    Sym(&close, "hdfsCloseFile");
    Sym(&pread, "hdfsPread");
    Sym(&write, "hdfsWrite");
    Sym(&path_info, "hdfsGetPathInfo");
    Sym(&list, "hdfsListDirectory");
    Sym(&free_info, "hdfsFreeFileInfo");
    Sym(&hosts, "hdfsGetHosts");
    Sym(&free_hosts, "hdfsFreeHosts");
    Sym(&exists, "hdfsExists");
    Sym(&mkdir, "hdfsCreateDirectory");
    Sym(&rename, "hdfsRename");
    Sym(&del, "hdfsDelete");
  }
};

class NativeHdfs : public FileSystem {
 public:
  NativeHdfs(const std::string& host, int port) : lib_(LibHdfs3::Get()), authority_(host + ":" + std::to_string(port)) {
    MINIPS_CHECK(lib_.error.empty(), lib_.error);
    fs_ = lib_.connect(host.c_str(), (uint16_t)port);
    MINIPS_CHECK(fs_ != nullptr, "hdfsConnect(" << authority_ << ") failed");
  }
  ~NativeHdfs() override { lib_.disconnect(fs_); }
  std::string Name() const override { return "hdfs://" + authority_; }
  FileStat Info(const std::string& url, const HdfsFileInfoAbi& i) {
    return FileStat{url, (uint64_t)i.mSize, (uint64_t)i.mBlockSize, i.mKind == 'D'};
  }
  FileStat Stat(const std::string& url) override {
    HdfsFileInfoAbi* i = lib_.path_info(fs_, ParseUrl(url).path.c_str());
    MINIPS_CHECK(i != nullptr, "no such file " << url);
    FileStat f = Info(url, *i);
    lib_.free_info(i, 1);
    return f;
  }
  bool Exists(const std::string& url) override { return lib_.exists(fs_, ParseUrl(url).path.c_str()) == 0; }
  std::vector<FileStat> List(const std::string& url) override {
    FileStat top = Stat(url);
    if (!top.is_dir) return {top};
    int n = 0;
    HdfsFileInfoAbi* l = lib_.list(fs_, ParseUrl(url).path.c_str(), &n);
    std::vector<FileStat> out;
    for (int i = 0; i < n; ++i) {
      if (l[i].mKind == 'D') continue;
      std::string name = l[i].mName;
      name = name.substr(name.find_last_of('/') + 1);
      out.push_back(Info(JoinPath(url, name), l[i]));
    }
    if (l) lib_.free_info(l, n);
    std::sort(out.begin(), out.end(), [](const FileStat& a, const FileStat& b) { return a.url < b.url; });
    return out;
  }
  std::vector<BlockLocation> Locations(const FileStat& f) override {
    std::vector<BlockLocation> out;
    char*** h = lib_.hosts(fs_, ParseUrl(f.url).path.c_str(), 0, (int64_t)f.size);
    const uint64_t bs = f.block_size ? f.block_size : std::max<uint64_t>(f.size, 1);
    for (uint64_t b = 0; h && h[b]; ++b) {
      BlockLocation l{b * bs, std::min(bs, f.size - std::min(f.size, b * bs)), {}};
      for (int r = 0; h[b][r]; ++r) l.hosts.push_back(h[b][r]);
      out.push_back(std::move(l));
    }
    if (h) lib_.free_hosts(h);
    return out;
  }
  class File : public RandomAccessFile {
   public:
    File(NativeHdfs* fs, void* f, uint64_t size) : fs_(fs), f_(f), size_(size) {}
    ~File() override { fs_->lib_.close(fs_->fs_, f_); }
    uint64_t Size() const override { return size_; }
    size_t ReadAt(uint64_t off, char* buf, size_t n) override {
      size_t got = 0;
      while (got < n && off + got < size_) {
        const int32_t want = (int32_t)std::min<size_t>(n - got, 1 << 30);
        int32_t r = fs_->lib_.pread(fs_->fs_, f_, (int64_t)(off + got), buf + got, want);
        MINIPS_CHECK(r >= 0, "hdfsPread failed");
        if (r == 0) break;
        got += (size_t)r;
      }
      g_remote_bytes += got;
      return got;
    }

   private:
    NativeHdfs* fs_;
    void* f_;
    uint64_t size_;
  };
  std::unique_ptr<RandomAccessFile> OpenRead(const std::string& url) override {
    FileStat st = Stat(url);
    void* f = lib_.open(fs_, ParseUrl(url).path.c_str(), O_RDONLY, 0, 0, 0);
    MINIPS_CHECK(f != nullptr, "hdfsOpenFile " << url);
    return std::unique_ptr<RandomAccessFile>(new File(this, f, st.size));
  }
  class Out : public WritableFile {
   public:
    Out(NativeHdfs* fs, void* f) : fs_(fs), f_(f) {}
    ~Out() override {
      if (f_) fs_->lib_.close(fs_->fs_, f_);
    }
    void Append(const char* d, size_t n) override {
      while (n > 0) {
        int32_t w = fs_->lib_.write(fs_->fs_, f_, d, (int32_t)std::min<size_t>(n, 1 << 30));
        MINIPS_CHECK(w > 0, "hdfsWrite failed");
        d += w;
        n -= (size_t)w;
      }
    }
    void Close() override {
      if (!f_) return;
      const int rc = fs_->lib_.close(fs_->fs_, f_);
      f_ = nullptr;
      MINIPS_CHECK(rc == 0, "hdfsCloseFile failed");
    }

   private:
    NativeHdfs* fs_;
    void* f_;
  };
  std::unique_ptr<WritableFile> OpenWrite(const std::string& url) override {
    void* f = lib_.open(fs_, ParseUrl(url).path.c_str(), O_WRONLY | O_CREAT, 0, 0, 0);
    MINIPS_CHECK(f != nullptr, "hdfsOpenFile(write) " << url);
    return std::unique_ptr<WritableFile>(new Out(this, f));
  }
  void MakeDirs(const std::string& url) override { lib_.mkdir(fs_, ParseUrl(url).path.c_str()); }
  void Rename(const std::string& a, const std::string& b) override {
    MINIPS_CHECK(lib_.rename(fs_, ParseUrl(a).path.c_str(), ParseUrl(b).path.c_str()) == 0, "hdfsRename " << a);
  }
  void Remove(const std::string& url) override { lib_.del(fs_, ParseUrl(url).path.c_str(), 1); }

 private:
  LibHdfs3& lib_;
  std::string authority_;
  void* fs_ = nullptr;
};

}  // namespace

std::string Url::ToString() const {
  if (scheme.empty()) return path;
  return scheme + "://" + host + (port ? ":" + std::to_string(port) : "") + path + (query.empty() ? "" : "?" + query);
}

Url ParseUrl(const std::string& s) {
  Url u;
  const size_t sep = s.find("://");
  if (sep == std::string::npos) {
    u.path = s;
    return u;
  }
  u.scheme = s.substr(0, sep);
  std::string rest = s.substr(sep + 3);
  const size_t slash = rest.find('/');
  std::string auth = slash == std::string::npos ? rest : rest.substr(0, slash);
  std::string path = slash == std::string::npos ? "/" : rest.substr(slash);
  const size_t q = path.find('?');
  if (q != std::string::npos) {
    u.query = path.substr(q + 1);
    path = path.substr(0, q);
  }
  const size_t colon = auth.rfind(':');
  if (colon != std::string::npos) {
    u.host = auth.substr(0, colon);
    u.port = std::atoi(auth.c_str() + colon + 1);
  } else {
    u.host = auth;
  }
  u.path = path;
  MINIPS_CHECK(u.scheme == "file" || !u.host.empty() || u.scheme.empty(), "URL without a host: " << s);
  return u;
}

bool IsLocalUrl(const std::string& url) {
  const Url u = ParseUrl(url);
  return u.scheme.empty() || u.scheme == "file";
}

std::string LocalHostName() {
  if (const char* h = std::getenv("MINIPS_HOSTNAME")) return h;  // tests / multi-homed hosts
  char buf[256] = {0};
  if (::gethostname(buf, sizeof(buf) - 1) != 0) return "localhost";
  return buf;
}

bool LibHdfs3Available(std::string* why) {
  LibHdfs3& l = LibHdfs3::Get();
  if (why) *why = l.error;
  return l.error.empty();
}

FileSystem& FileSystem::For(const std::string& url) {
  static std::mutex mu;
  static std::map<std::string, std::unique_ptr<FileSystem>> pool;  // scheme://authority -> fs
  const Url u = ParseUrl(url);
  std::lock_guard<std::mutex> lk(mu);
  if (u.scheme.empty() || u.scheme == "file") {
    auto& fs = pool["local"];
    if (!fs) fs.reset(new LocalFs());
    return *fs;
  }
  const std::string key = u.scheme + "://" + u.host + ":" + std::to_string(u.port);
  auto& fs = pool[key];
  if (fs) return *fs;
  if (u.scheme == "webhdfs") {
    fs.reset(new WebHdfs(u.host, u.port ? u.port : 9870));
  } else if (u.scheme == "hdfs") {
    const char* http = std::getenv("MINIPS_HDFS_HTTP_PORT");
    if (http && *http) {
      fs.reset(new WebHdfs(u.host, std::atoi(http)));
    } else {
      fs.reset(new NativeHdfs(u.host, u.port ? u.port : 8020));
    }
  } else {
    MINIPS_CHECK(false, "unsupported URL scheme '" << u.scheme << "' in " << url);
  }
  return *fs;
}

std::string ReadFileToString(const std::string& url) {
  auto f = FileSystem::For(url).OpenRead(url);
  std::string s(f->Size(), '\0');
  const size_t got = s.empty() ? 0 : f->ReadAt(0, &s[0], s.size());
  s.resize(got);
  return s;
}

void WriteStringToFile(const std::string& url, const std::string& data) {
  auto f = FileSystem::For(url).OpenWrite(url);
  f->Append(data.data(), data.size());
  f->Close();
}

uint64_t RemoteBytesRead() { return g_remote_bytes.load(); }

FsReadBuf::int_type FsReadBuf::underflow() {
  if (gptr() < egptr()) return traits_type::to_int_type(*gptr());
  base_ += (uint64_t)(egptr() - eback());
  const size_t got = f_->ReadAt(base_, buf_.data(), buf_.size());
  setg(buf_.data(), buf_.data(), buf_.data() + got);
  return got ? traits_type::to_int_type(*gptr()) : traits_type::eof();
}

FsReadBuf::pos_type FsReadBuf::seekoff(off_type off, std::ios_base::seekdir dir, std::ios_base::openmode) {
  const uint64_t cur = base_ + (uint64_t)(gptr() - eback());
  int64_t target = dir == std::ios_base::beg ? off : dir == std::ios_base::cur ? (int64_t)cur + off
                                                                              : (int64_t)f_->Size() + off;
  if (target < 0 || (uint64_t)target > f_->Size()) return pos_type(off_type(-1));
  if ((uint64_t)target >= base_ && (uint64_t)target < base_ + (uint64_t)(egptr() - eback())) {
    setg(eback(), eback() + (target - (int64_t)base_), egptr());
  } else {
    base_ = (uint64_t)target;
    setg(buf_.data(), buf_.data(), buf_.data());
  }
  return pos_type(target);
}

FsWriteBuf::FsWriteBuf(std::unique_ptr<WritableFile> f, size_t buf) : f_(std::move(f)), buf_(buf) {
  setp(buf_.data(), buf_.data() + buf_.size());
}

FsWriteBuf::~FsWriteBuf() { Close(); }

bool FsWriteBuf::Drain() {
  const size_t n = (size_t)(pptr() - pbase());
  if (n && !failed_) {
    try {
      f_->Append(pbase(), n);
    } catch (const std::exception&) {
      failed_ = true;
    }
  }
  setp(buf_.data(), buf_.data() + buf_.size());
  return !failed_;
}

FsWriteBuf::int_type FsWriteBuf::overflow(int_type c) {
  if (!Drain()) return traits_type::eof();
  if (!traits_type::eq_int_type(c, traits_type::eof())) {
    *pptr() = traits_type::to_char_type(c);
    pbump(1);
  }
  return traits_type::not_eof(c);
}

int FsWriteBuf::sync() { return Drain() ? 0 : -1; }

bool FsWriteBuf::Close() {
  if (!f_) return !failed_;
  Drain();
  try {
    f_->Close();
  } catch (const std::exception&) {
    failed_ = true;
  }
  f_.reset();
  return !failed_;
}

GeneralIfstream::GeneralIfstream(const std::string& url) : std::istream(nullptr) {
  try {
    sb_.reset(new FsReadBuf(FileSystem::For(url).OpenRead(url)));
    rdbuf(sb_.get());
  } catch (const std::exception&) {
    setstate(std::ios::failbit);
  }
}

GeneralOfstream::GeneralOfstream(const std::string& url) : std::ostream(nullptr) {
  try {
    sb_.reset(new FsWriteBuf(FileSystem::For(url).OpenWrite(url)));
    rdbuf(sb_.get());
  } catch (const std::exception&) {
    setstate(std::ios::failbit);
  }
}

GeneralOfstream::~GeneralOfstream() {
  if (sb_) sb_->Close();
}

void GeneralOfstream::close() {
  if (sb_ && !sb_->Close()) setstate(std::ios::badbit);
}

}  // namespace minips
