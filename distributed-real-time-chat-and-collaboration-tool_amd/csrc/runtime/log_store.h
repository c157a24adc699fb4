// Append-only durable Raft log.
//
// The reference rewrites the WHOLE log pickle on every append
// (server/raft_node.py:198-214, survey quirk Q5: O(history) per write, no
// fsync).  This store appends one CRC-checked record per entry and keeps an
// in-memory offset index, so an append is O(entry) and truncation (Raft
// conflict resolution) is an ftruncate.  On open, records are scanned and the
// file is cut at the first torn/corrupt record (crash during append).
//
// Record: u32 magic | u32 body_len | body | u32 crc32(body)
//   body: i64 term | u32 cmd_len | cmd | u32 data_len | data
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace drtc {

struct LogRecord {
  int64_t term;
  std::string command;
  std::string data;
};

class LogStore {
 public:
  explicit LogStore(const std::string& path, bool fsync_each = false);
  ~LogStore();
  LogStore(const LogStore&) = delete;
  LogStore& operator=(const LogStore&) = delete;

  int64_t size() const { return (int64_t)offsets_.size(); }
  // Returns the 0-based index of the appended entry.
  int64_t append(int64_t term, const std::string& command, const std::string& data);
  LogRecord get(int64_t index) const;
  int64_t term_at(int64_t index) const;
  // Drop entries [index, size).
  void truncate_from(int64_t index);
  void sync();
  void close();

 private:
  std::string path_;
  int fd_ = -1;
  bool fsync_each_;
  uint64_t end_ = 0;
  std::vector<uint64_t> offsets_;
  std::vector<int64_t> terms_;
};

uint32_t crc32(const uint8_t* data, size_t n, uint32_t crc = 0);

}  // namespace drtc
