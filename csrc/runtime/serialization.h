// BinStream: byte-stream (de)serialisation for control-plane payloads and checkpoint metadata
// (reference base/serialization.{hpp,cpp}: << / >> for PODs, strings, vectors, maps, pairs,
// smart pointers, and any type with serialize(BinStream&) const / deserialize(BinStream&)).
#pragma once

#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <type_traits>
#include <unordered_map>
#include <utility>
#include <vector>

#include "base.h"

namespace minips {

class BinStream;

template <typename T, typename = void>
struct has_serialize : std::false_type {};
template <typename T>
struct has_serialize<T, std::void_t<decltype(std::declval<const T&>().serialize(std::declval<BinStream&>())),
                                    decltype(std::declval<T&>().deserialize(std::declval<BinStream&>()))>>
    : std::true_type {};

class BinStream {
 public:
  BinStream() = default;
  explicit BinStream(std::vector<char> v) : buf_(std::move(v)) {}
  BinStream(const char* data, size_t n) : buf_(data, data + n) {}

  size_t size() const { return buf_.size() - front_; }
  const char* data() const { return buf_.data() + front_; }
  const std::vector<char>& buffer() const { return buf_; }
  void clear() {
    buf_.clear();
    front_ = 0;
  }
  void append(const void* p, size_t n) {
    const char* c = static_cast<const char*>(p);
    buf_.insert(buf_.end(), c, c + n);
  }
  void pop_front(void* p, size_t n) {
    MINIPS_CHECK(front_ + n <= buf_.size(), "BinStream underflow: need " << n << ", have " << size());
    std::memcpy(p, buf_.data() + front_, n);
    front_ += n;
  }
  SArray<char> ToSArray() const {
    SArray<char> s(size());
    if (size()) std::memcpy(s.data(), data(), size());
    return s;
  }
  static BinStream FromSArray(const SArray<char>& s) { return BinStream(s.data(), s.size()); }

 private:
  std::vector<char> buf_;
  size_t front_ = 0;
};

// ---- PODs and user types
template <typename T>
std::enable_if_t<std::is_trivially_copyable<T>::value && !has_serialize<T>::value, BinStream&> operator<<(
    BinStream& s, const T& v) {
  s.append(&v, sizeof(T));
  return s;
}
template <typename T>
std::enable_if_t<std::is_trivially_copyable<T>::value && !has_serialize<T>::value, BinStream&> operator>>(
    BinStream& s, T& v) {
  s.pop_front(&v, sizeof(T));
  return s;
}
template <typename T>
std::enable_if_t<has_serialize<T>::value, BinStream&> operator<<(BinStream& s, const T& v) {
  v.serialize(s);
  return s;
}
template <typename T>
std::enable_if_t<has_serialize<T>::value, BinStream&> operator>>(BinStream& s, T& v) {
  v.deserialize(s);
  return s;
}

// ---- strings
inline BinStream& operator<<(BinStream& s, const std::string& v) {
  s << (uint64_t)v.size();
  s.append(v.data(), v.size());
  return s;
}
inline BinStream& operator>>(BinStream& s, std::string& v) {
  uint64_t n;
  s >> n;
  v.resize(n);
  if (n) s.pop_front(&v[0], n);
  return s;
}

// ---- pairs
template <typename A, typename B>
BinStream& operator<<(BinStream& s, const std::pair<A, B>& p) {
  return s << p.first << p.second;
}
template <typename A, typename B>
BinStream& operator>>(BinStream& s, std::pair<A, B>& p) {
  return s >> p.first >> p.second;
}

// ---- vectors (bulk copy for trivially copyable elements)
template <typename T>
BinStream& operator<<(BinStream& s, const std::vector<T>& v) {
  s << (uint64_t)v.size();
  if constexpr (std::is_trivially_copyable<T>::value && !has_serialize<T>::value) {
    if (!v.empty()) s.append(v.data(), v.size() * sizeof(T));
  } else {
    for (const auto& e : v) s << e;
  }
  return s;
}
template <typename T>
BinStream& operator>>(BinStream& s, std::vector<T>& v) {
  uint64_t n;
  s >> n;
  v.resize(n);
  if constexpr (std::is_trivially_copyable<T>::value && !has_serialize<T>::value) {
    if (n) s.pop_front(v.data(), n * sizeof(T));
  } else {
    for (auto& e : v) s >> e;
  }
  return s;
}

// ---- SArray (bulk copy)
template <typename T>
BinStream& operator<<(BinStream& s, const SArray<T>& v) {
  s << (uint64_t)v.size();
  if (v.size()) s.append(v.data(), v.size() * sizeof(T));
  return s;
}
template <typename T>
BinStream& operator>>(BinStream& s, SArray<T>& v) {
  uint64_t n;
  s >> n;
  v.resize(n);
  if (n) s.pop_front(v.data(), n * sizeof(T));
  return s;
}

// ---- maps
template <typename K, typename V>
BinStream& operator<<(BinStream& s, const std::map<K, V>& m) {
  s << (uint64_t)m.size();
  for (const auto& kv : m) s << kv.first << kv.second;
  return s;
}
template <typename K, typename V>
BinStream& operator>>(BinStream& s, std::map<K, V>& m) {
  uint64_t n;
  s >> n;
  m.clear();
  for (uint64_t i = 0; i < n; ++i) {
    K k;
    V v;
    s >> k >> v;
    m.emplace(std::move(k), std::move(v));
  }
  return s;
}
template <typename K, typename V>
BinStream& operator<<(BinStream& s, const std::unordered_map<K, V>& m) {
  s << (uint64_t)m.size();
  for (const auto& kv : m) s << kv.first << kv.second;
  return s;
}
template <typename K, typename V>
BinStream& operator>>(BinStream& s, std::unordered_map<K, V>& m) {
  uint64_t n;
  s >> n;
  m.clear();
  for (uint64_t i = 0; i < n; ++i) {
    K k;
    V v;
    s >> k >> v;
    m.emplace(std::move(k), std::move(v));
  }
  return s;
}

// ---- smart pointers (null flag + value)
template <typename T>
BinStream& operator<<(BinStream& s, const std::shared_ptr<T>& p) {
  s << (uint8_t)(p ? 1 : 0);
  if (p) s << *p;
  return s;
}
template <typename T>
BinStream& operator>>(BinStream& s, std::shared_ptr<T>& p) {
  uint8_t f;
  s >> f;
  if (f) {
    p = std::make_shared<T>();
    s >> *p;
  } else {
    p.reset();
  }
  return s;
}
template <typename T>
BinStream& operator<<(BinStream& s, const std::unique_ptr<T>& p) {
  s << (uint8_t)(p ? 1 : 0);
  if (p) s << *p;
  return s;
}
template <typename T>
BinStream& operator>>(BinStream& s, std::unique_ptr<T>& p) {
  uint8_t f;
  s >> f;
  if (f) {
    p.reset(new T());
    s >> *p;
  } else {
    p.reset();
  }
  return s;
}

}  // namespace minips
