#include "log_store.h"

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstring>
#include <stdexcept>

namespace drtc {

namespace {
constexpr uint32_t kMagic = 0x52414654;  // "RAFT"

uint32_t crc_table_entry(uint32_t c) {
  for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
  return c;
}

struct CrcTable {
  uint32_t t[256];
  CrcTable() {
    for (uint32_t i = 0; i < 256; ++i) t[i] = crc_table_entry(i);
  }
};
const CrcTable& table() {
  static CrcTable tb;
  return tb;
}

bool read_full(int fd, void* buf, size_t n, uint64_t off) {
  auto* p = (uint8_t*)buf;
  while (n) {
    ssize_t r = pread(fd, p, n, (off_t)off);
    if (r <= 0) return false;
    p += r;
    n -= (size_t)r;
    off += (uint64_t)r;
  }
  return true;
}

void write_full(int fd, const void* buf, size_t n, uint64_t off) {
  auto* p = (const uint8_t*)buf;
  while (n) {
    ssize_t r = pwrite(fd, p, n, (off_t)off);
    if (r <= 0) throw std::runtime_error("LogStore: write failed");
    p += r;
    n -= (size_t)r;
    off += (uint64_t)r;
  }
}

void put_u32(std::string& s, uint32_t v) { s.append((const char*)&v, 4); }
void put_i64(std::string& s, int64_t v) { s.append((const char*)&v, 8); }
}  // namespace

uint32_t crc32(const uint8_t* data, size_t n, uint32_t crc) {
  crc = ~crc;
  const auto& tb = table();
  for (size_t i = 0; i < n; ++i) crc = tb.t[(crc ^ data[i]) & 0xff] ^ (crc >> 8);
  return ~crc;
}

LogStore::LogStore(const std::string& path, bool fsync_each) : path_(path), fsync_each_(fsync_each) {
  fd_ = ::open(path.c_str(), O_RDWR | O_CREAT, 0644);
  if (fd_ < 0) throw std::runtime_error("LogStore: cannot open " + path);
  struct stat st;
  fstat(fd_, &st);
  const uint64_t fsize = (uint64_t)st.st_size;
  uint64_t off = 0;
  std::string body;
  while (off + 8 <= fsize) {
    uint32_t hdr[2];
    if (!read_full(fd_, hdr, 8, off) || hdr[0] != kMagic) break;
    const uint64_t blen = hdr[1];
    if (off + 8 + blen + 4 > fsize || blen < 16) break;
    body.resize(blen);
    uint32_t crc;
    if (!read_full(fd_, body.data(), blen, off + 8) || !read_full(fd_, &crc, 4, off + 8 + blen)) break;
    if (crc32((const uint8_t*)body.data(), blen) != crc) break;
    int64_t term;
    std::memcpy(&term, body.data(), 8);
    offsets_.push_back(off);
    terms_.push_back(term);
    off += 8 + blen + 4;
  }
  end_ = off;
  if (end_ != fsize) {
    if (ftruncate(fd_, (off_t)end_) != 0) throw std::runtime_error("LogStore: truncate failed");
  }
}

LogStore::~LogStore() { close(); }

void LogStore::close() {
  if (fd_ >= 0) {
    ::fsync(fd_);
    ::close(fd_);
    fd_ = -1;
  }
}

int64_t LogStore::append(int64_t term, const std::string& command, const std::string& data) {
  if (fd_ < 0) throw std::runtime_error("LogStore: closed");
  std::string body;
  body.reserve(16 + command.size() + data.size());
  put_i64(body, term);
  put_u32(body, (uint32_t)command.size());
  body += command;
  put_u32(body, (uint32_t)data.size());
  body += data;
  std::string rec;
  rec.reserve(body.size() + 12);
  put_u32(rec, kMagic);
  put_u32(rec, (uint32_t)body.size());
  rec += body;
  put_u32(rec, crc32((const uint8_t*)body.data(), body.size()));
  write_full(fd_, rec.data(), rec.size(), end_);
  offsets_.push_back(end_);
  terms_.push_back(term);
  end_ += rec.size();
  if (fsync_each_) ::fdatasync(fd_);
  return (int64_t)offsets_.size() - 1;
}

LogRecord LogStore::get(int64_t index) const {
  if (index < 0 || index >= size()) throw std::out_of_range("LogStore: index out of range");
  uint32_t hdr[2];
  const uint64_t off = offsets_[index];
  if (!read_full(fd_, hdr, 8, off)) throw std::runtime_error("LogStore: read failed");
  std::string body(hdr[1], '\0');
  if (!read_full(fd_, body.data(), body.size(), off + 8)) throw std::runtime_error("LogStore: read failed");
  LogRecord r;
  std::memcpy(&r.term, body.data(), 8);
  uint32_t cl;
  std::memcpy(&cl, body.data() + 8, 4);
  r.command.assign(body.data() + 12, cl);
  uint32_t dl;
  std::memcpy(&dl, body.data() + 12 + cl, 4);
  r.data.assign(body.data() + 16 + cl, dl);
  return r;
}

int64_t LogStore::term_at(int64_t index) const {
  if (index < 0 || index >= size()) return 0;
  return terms_[index];
}

void LogStore::truncate_from(int64_t index) {
  if (index < 0) index = 0;
  if (index >= size()) return;
  end_ = offsets_[index];
  offsets_.resize(index);
  terms_.resize(index);
  if (ftruncate(fd_, (off_t)end_) != 0) throw std::runtime_error("LogStore: truncate failed");
  if (fsync_each_) ::fdatasync(fd_);
}

void LogStore::sync() {
  if (fd_ >= 0) ::fdatasync(fd_);
}

}  // namespace drtc
