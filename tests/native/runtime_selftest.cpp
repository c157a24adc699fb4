// Host-side self-test of the native CPU runtime (csrc/runtime), built with
// -fsanitize=address,undefined by tests/test_native_sanitizers.py (SURVEY §5
// "Race detection / sanitizers": ASan/UBSan builds for the C++ extensions).
//
//  * bcrypt: hashes of random passwords/salts equal libxcrypt's crypt_rn()
//    output (costs 4-5, $2a$ and $2b$, 0..80-byte passwords incl. the
//    72-byte truncation), checkpw accepts/rejects correctly.
//  * BlockAllocator: randomized alloc / incref / free against a shadow
//    model; double free and out-of-range ids throw.
//  * LogStore: append / get / truncate / reopen round trips and torn-tail
//    recovery after cutting the file at every byte of the last record.
#include <crypt.h>
#include <fcntl.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>
#include <map>
#include <random>
#include <stdexcept>
#include <string>
#include <vector>

#include "bcrypt.h"
#include "block_allocator.h"
#include "log_store.h"

static int failures = 0;
#define CHECK(c)                                                         \
  do {                                                                   \
    if (!(c)) {                                                          \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++failures;                                                        \
    }                                                                    \
  } while (0)

static void test_bcrypt(std::mt19937& rng) {
  for (int it = 0; it < 24; ++it) {
    uint8_t salt[16];
    for (auto& b : salt) b = (uint8_t)rng();
    const int cost = 4 + it % 2;
    const char minor = it % 3 == 0 ? 'a' : 'b';
    const std::string settings = drtc::bcrypt_gensalt(cost, salt, minor);
    std::string pw;
    const int n = (int)(rng() % 81);
    for (int i = 0; i < n; ++i) pw.push_back((char)(1 + rng() % 255));
    const std::string mine = drtc::bcrypt_hashpw(pw, settings);
    crypt_data cd;
    std::memset(&cd, 0, sizeof(cd));
    const char* ref = crypt_rn(pw.c_str(), settings.c_str(), &cd, sizeof(cd));
    CHECK(ref != nullptr && mine == std::string(ref));
    CHECK(drtc::bcrypt_checkpw(pw, mine));
    if (pw.size() < 72) CHECK(!drtc::bcrypt_checkpw(pw + "x", mine));  // bytes >72 are ignored
    else CHECK(drtc::bcrypt_checkpw(pw + "x", mine));
  }
  bool threw = false;
  try {
    drtc::bcrypt_hashpw("pw", "$2b$99$short");
  } catch (const std::exception&) {
    threw = true;
  }
  CHECK(threw);
}

static void test_allocator(std::mt19937& rng) {
  drtc::BlockAllocator a(257, 1);
  std::map<int32_t, int> ref;  // shadow refcounts
  for (int it = 0; it < 20000; ++it) {
    const int op = rng() % 4;
    if (op == 0 && a.can_allocate(3)) {
      for (int32_t b : a.allocate(3)) {
        CHECK(b >= 1 && b < 257 && ref[b] == 0);
        ref[b] = 1;
      }
    } else if (op == 1 && a.can_allocate(1)) {
      const int32_t b = a.allocate_one();
      CHECK(ref[b] == 0);
      ref[b] = 1;
    } else if (!ref.empty()) {
      auto itb = ref.begin();
      std::advance(itb, rng() % ref.size());
      const int32_t b = itb->first;
      if (op == 2) {
        a.incref({b});
        ++itb->second;
      } else {
        a.free({b});
        if (--itb->second == 0) ref.erase(itb);
      }
      if (ref.count(b)) CHECK(a.refcount(b) == ref[b]);
    }
    CHECK(a.num_used() == (int32_t)ref.size());
  }
  bool threw = false;
  try {
    a.refcount(0);  // reserved
  } catch (const std::out_of_range&) {
    threw = true;
  }
  CHECK(threw);
  const int32_t b = a.allocate_one();
  a.free({b});
  threw = false;
  try {
    a.free({b});
  } catch (const std::runtime_error&) {
    threw = true;
  }
  CHECK(threw);
}

static void test_log_store(std::mt19937& rng, const std::string& dir) {
  const std::string path = dir + "/selftest.log";
  std::remove(path.c_str());
  std::vector<drtc::LogRecord> model;
  {
    drtc::LogStore s(path);
    for (int i = 0; i < 300; ++i) {
      drtc::LogRecord r{(int64_t)(i / 7), "CMD" + std::to_string(i % 8),
                        std::string(rng() % 300, (char)('a' + i % 26))};
      CHECK(s.append(r.term, r.command, r.data) == (int64_t)model.size());
      model.push_back(r);
      if (i % 50 == 49) {
        const int64_t cut = (int64_t)model.size() - 1 - (int64_t)(rng() % 5);
        s.truncate_from(cut);
        model.resize(cut);
      }
    }
    for (size_t i = 0; i < model.size(); ++i) {
      const auto g = s.get((int64_t)i);
      CHECK(g.term == model[i].term && g.command == model[i].command && g.data == model[i].data);
    }
    s.sync();
  }
  {
    drtc::LogStore s(path);  // reopen: full scan
    CHECK(s.size() == (int64_t)model.size());
    for (size_t i = 0; i < model.size(); i += 13) CHECK(s.get((int64_t)i).data == model[i].data);
  }
  // torn tail: cut the file inside the last record at every byte offset
  int fd = ::open(path.c_str(), O_RDONLY);
  const off_t full = ::lseek(fd, 0, SEEK_END);
  ::close(fd);
  const drtc::LogRecord& last = model.back();
  const off_t rec = 4 + 4 + 8 + 4 + (off_t)last.command.size() + 4 + (off_t)last.data.size() + 4;
  for (off_t cut = full - rec + 1; cut < full; cut += 1 + rec / 40) {
    CHECK(::truncate(path.c_str(), cut) == 0);
    drtc::LogStore s(path);
    CHECK(s.size() == (int64_t)model.size() - 1);
    CHECK(s.get(s.size() - 1).data == model[model.size() - 2].data);
    s.append(last.term, last.command, last.data);  // heal for the next cut
  }
  std::remove(path.c_str());
}

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp";
  std::mt19937 rng(1234);
  test_bcrypt(rng);
  test_allocator(rng);
  test_log_store(rng, dir);
  if (failures) {
    std::fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  std::printf("runtime selftest OK\n");
  return 0;
}
