// bcrypt ($2a$/$2b$/$2y$, EksBlowfish) — native password hashing for the chat
// service's Signup/Login (the reference uses pyca/bcrypt, a Rust extension:
// server/raft_node.py:437,1411,1450).  Output is byte-compatible with it,
// so hashes stored in users.pkl / the Raft log verify across both stacks.
#pragma once
#include <cstdint>
#include <string>

namespace drtc {

// Hash `password` with the settings string `salt` ("$2b$12$<22 chars>...").
// Throws std::invalid_argument on a malformed settings string.
std::string bcrypt_hashpw(const std::string& password, const std::string& salt);

// Constant-time comparison of bcrypt_hashpw(password, hashed) with hashed.
bool bcrypt_checkpw(const std::string& password, const std::string& hashed);

// "$2b$<cost>$" + 22 salt chars from 16 caller-provided random bytes.
std::string bcrypt_gensalt(int cost, const uint8_t random16[16], char minor = 'b');

}  // namespace drtc
