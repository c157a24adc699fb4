// EksBlowfish / bcrypt, written from the published algorithm (Provos &
// Mazieres 1999; OpenBSD $2b$ key-length rules).
#include "bcrypt.h"

#include <cstring>
#include <stdexcept>

#include "blowfish_init.h"

namespace drtc {
namespace {

constexpr char kB64[] = "./ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789";

struct Blowfish {
  uint32_t P[18];
  uint32_t S[4][256];

  void init() {
    std::memcpy(P, kBlowfishP, sizeof(P));
    std::memcpy(S, kBlowfishS, sizeof(S));
  }
  inline uint32_t F(uint32_t x) const {
    return ((S[0][x >> 24] + S[1][(x >> 16) & 0xff]) ^ S[2][(x >> 8) & 0xff]) +
           S[3][x & 0xff];
  }
  inline void encipher(uint32_t& xl, uint32_t& xr) const {
    uint32_t L = xl ^ P[0], R = xr;
    for (int i = 1; i <= 16; i += 2) {
      R ^= F(L) ^ P[i];
      L ^= F(R) ^ P[i + 1];
    }
    xl = R ^ P[17];
    xr = L;
  }
};

inline uint32_t stream_word(const uint8_t* data, size_t len, size_t& pos) {
  uint32_t w = 0;
  for (int i = 0; i < 4; ++i) {
    if (pos >= len) pos = 0;
    w = (w << 8) | data[pos++];
  }
  return w;
}

// ExpandKey(state, salt, key); salt == nullptr is the "Expand0State" form.
void expand_key(Blowfish& bf, const uint8_t* salt, size_t salt_len, const uint8_t* key,
                size_t key_len) {
  size_t kp = 0;
  for (int i = 0; i < 18; ++i) bf.P[i] ^= stream_word(key, key_len, kp);
  uint32_t L = 0, R = 0;
  size_t sp = 0;
  auto step = [&](uint32_t& a, uint32_t& b) {
    if (salt) {
      L ^= stream_word(salt, salt_len, sp);
      R ^= stream_word(salt, salt_len, sp);
    }
    bf.encipher(L, R);
    a = L;
    b = R;
  };
  for (int i = 0; i < 18; i += 2) step(bf.P[i], bf.P[i + 1]);
  for (int s = 0; s < 4; ++s)
    for (int k = 0; k < 256; k += 2) step(bf.S[s][k], bf.S[s][k + 1]);
}

std::string b64_encode(const uint8_t* d, size_t n) {
  std::string out;
  size_t i = 0;
  while (i < n) {
    uint32_t c1 = d[i++];
    out.push_back(kB64[c1 >> 2]);
    c1 = (c1 & 0x03) << 4;
    if (i >= n) { out.push_back(kB64[c1]); break; }
    uint32_t c2 = d[i++];
    c1 |= (c2 >> 4) & 0x0f;
    out.push_back(kB64[c1]);
    c1 = (c2 & 0x0f) << 2;
    if (i >= n) { out.push_back(kB64[c1]); break; }
    c2 = d[i++];
    c1 |= (c2 >> 6) & 0x03;
    out.push_back(kB64[c1]);
    out.push_back(kB64[c2 & 0x3f]);
  }
  return out;
}

int b64_index(char c) {
  const char* p = std::strchr(kB64, c);
  return (p && c) ? (int)(p - kB64) : -1;
}

// Decode exactly `n` bytes from the bcrypt-base64 string.
bool b64_decode(const char* s, uint8_t* out, size_t n) {
  size_t o = 0, i = 0;
  while (o < n) {
    int c1 = b64_index(s[i]), c2 = b64_index(s[i + 1]);
    if (c1 < 0 || c2 < 0) return false;
    out[o++] = (uint8_t)((c1 << 2) | ((c2 & 0x30) >> 4));
    if (o >= n) break;
    int c3 = b64_index(s[i + 2]);
    if (c3 < 0) return false;
    out[o++] = (uint8_t)(((c2 & 0x0f) << 4) | ((c3 & 0x3c) >> 2));
    if (o >= n) break;
    int c4 = b64_index(s[i + 3]);
    if (c4 < 0) return false;
    out[o++] = (uint8_t)(((c3 & 0x03) << 6) | c4);
    i += 4;
  }
  return true;
}

}  // namespace

std::string bcrypt_hashpw(const std::string& password, const std::string& setting) {
  // "$2?$NN$" + 22 salt chars
  if (setting.size() < 29 || setting[0] != '$' || setting[1] != '2' || setting[3] != '$' ||
      setting[6] != '$')
    throw std::invalid_argument("invalid bcrypt salt");
  const char minor = setting[2];
  if (minor != 'a' && minor != 'b' && minor != 'y')
    throw std::invalid_argument("unsupported bcrypt version");
  if (setting[4] < '0' || setting[4] > '9' || setting[5] < '0' || setting[5] > '9')
    throw std::invalid_argument("invalid bcrypt cost");
  const int cost = (setting[4] - '0') * 10 + (setting[5] - '0');
  if (cost < 4 || cost > 31) throw std::invalid_argument("invalid bcrypt cost");
  uint8_t salt[16];
  if (!b64_decode(setting.c_str() + 7, salt, 16)) throw std::invalid_argument("invalid bcrypt salt");

  // Key = password bytes up to the first NUL, capped at 72, plus the NUL.
  size_t plen = strnlen(password.c_str(), password.size());
  if (plen > 72) plen = 72;
  uint8_t key[73];
  std::memcpy(key, password.data(), plen);
  key[plen] = 0;
  const size_t key_len = plen + 1;

  Blowfish bf;
  bf.init();
  expand_key(bf, salt, 16, key, key_len);
  const uint64_t rounds = 1ull << cost;
  for (uint64_t r = 0; r < rounds; ++r) {
    expand_key(bf, nullptr, 0, key, key_len);
    expand_key(bf, nullptr, 0, salt, 16);
  }
  static const char kMagic[] = "OrpheanBeholderScryDoubt";
  uint32_t cdata[6];
  size_t mp = 0;
  for (int i = 0; i < 6; ++i) cdata[i] = stream_word((const uint8_t*)kMagic, 24, mp);
  for (int i = 0; i < 64; ++i)
    for (int j = 0; j < 6; j += 2) bf.encipher(cdata[j], cdata[j + 1]);
  uint8_t ctext[24];
  for (int i = 0; i < 6; ++i) {
    ctext[4 * i + 0] = (uint8_t)(cdata[i] >> 24);
    ctext[4 * i + 1] = (uint8_t)(cdata[i] >> 16);
    ctext[4 * i + 2] = (uint8_t)(cdata[i] >> 8);
    ctext[4 * i + 3] = (uint8_t)(cdata[i]);
  }
  std::string out = setting.substr(0, 7);
  out += b64_encode(salt, 16);
  out += b64_encode(ctext, 23);
  std::memset(key, 0, sizeof(key));
  return out;
}

bool bcrypt_checkpw(const std::string& password, const std::string& hashed) {
  std::string h;
  try {
    h = bcrypt_hashpw(password, hashed);
  } catch (const std::exception&) {
    return false;
  }
  if (h.size() != hashed.size()) return false;
  unsigned char diff = 0;
  for (size_t i = 0; i < h.size(); ++i) diff |= (unsigned char)(h[i] ^ hashed[i]);
  return diff == 0;
}

std::string bcrypt_gensalt(int cost, const uint8_t random16[16], char minor) {
  if (cost < 4 || cost > 31) throw std::invalid_argument("invalid bcrypt cost");
  std::string s = "$2";
  s.push_back(minor);
  s.push_back('$');
  s.push_back((char)('0' + cost / 10));
  s.push_back((char)('0' + cost % 10));
  s.push_back('$');
  s += b64_encode(random16, 16);
  return s;
}

}  // namespace drtc
