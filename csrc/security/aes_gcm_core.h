// AES-256-GCM core over OpenSSL EVP (no Python dependency); see aes_gcm.cpp for the contract.
#pragma once
#include <openssl/evp.h>
#include <openssl/rand.h>

#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace pk_aes {

constexpr int kKeyLen = 32;
constexpr int kNonceLen = 12;
constexpr int kTagLen = 16;

struct CtxDeleter {
  void operator()(EVP_CIPHER_CTX* c) const { EVP_CIPHER_CTX_free(c); }
};
using CtxPtr = std::unique_ptr<EVP_CIPHER_CTX, CtxDeleter>;

inline void validate_key(const std::string& key) {
  if (key.size() != kKeyLen)
    throw std::invalid_argument("key length must be 32 bytes, got " + std::to_string(key.size()) + " bytes");
}

inline CtxPtr new_ctx() {
  CtxPtr c(EVP_CIPHER_CTX_new());
  if (!c) throw std::runtime_error("failed to create AES cipher: EVP_CIPHER_CTX_new");
  return c;
}

inline std::string seal(EVP_CIPHER_CTX* ctx, const std::string& key, const std::string& pt) {
  std::string out(kNonceLen + pt.size() + kTagLen, '\0');
  auto* o = reinterpret_cast<unsigned char*>(&out[0]);
  if (RAND_bytes(o, kNonceLen) != 1) throw std::runtime_error("failed to generate nonce: RAND_bytes");
  int len = 0, fin = 0;
  if (EVP_EncryptInit_ex(ctx, EVP_aes_256_gcm(), nullptr, nullptr, nullptr) != 1 ||
      EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_GCM_SET_IVLEN, kNonceLen, nullptr) != 1 ||
      EVP_EncryptInit_ex(ctx, nullptr, nullptr, reinterpret_cast<const unsigned char*>(key.data()), o) != 1)
    throw std::runtime_error("failed to create GCM cipher");
  if (!pt.empty() &&
      EVP_EncryptUpdate(ctx, o + kNonceLen, &len, reinterpret_cast<const unsigned char*>(pt.data()),
                        static_cast<int>(pt.size())) != 1)
    throw std::runtime_error("failed to encrypt");
  if (EVP_EncryptFinal_ex(ctx, o + kNonceLen + len, &fin) != 1) throw std::runtime_error("failed to encrypt");
  if (EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_GCM_GET_TAG, kTagLen, o + kNonceLen + pt.size()) != 1)
    throw std::runtime_error("failed to encrypt: tag");
  return out;
}

inline std::string open(EVP_CIPHER_CTX* ctx, const std::string& key, const std::string& in) {
  if (in.size() < static_cast<size_t>(kNonceLen))
    throw std::invalid_argument("ciphertext too short: " + std::to_string(in.size()) +
                                " bytes, expected at least " + std::to_string(kNonceLen) + " bytes");
  const auto* p = reinterpret_cast<const unsigned char*>(in.data());
  if (in.size() < static_cast<size_t>(kNonceLen + kTagLen))
    throw std::invalid_argument("failed to decrypt: cipher: message authentication failed");
  const size_t ct_len = in.size() - kNonceLen - kTagLen;
  std::string out(ct_len, '\0');
  auto* o = reinterpret_cast<unsigned char*>(&out[0]);
  int len = 0, fin = 0;
  if (EVP_DecryptInit_ex(ctx, EVP_aes_256_gcm(), nullptr, nullptr, nullptr) != 1 ||
      EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_GCM_SET_IVLEN, kNonceLen, nullptr) != 1 ||
      EVP_DecryptInit_ex(ctx, nullptr, nullptr, reinterpret_cast<const unsigned char*>(key.data()), p) != 1)
    throw std::runtime_error("failed to create GCM cipher");
  if (ct_len && EVP_DecryptUpdate(ctx, o, &len, p + kNonceLen, static_cast<int>(ct_len)) != 1)
    throw std::invalid_argument("failed to decrypt: cipher: message authentication failed");
  std::vector<unsigned char> tag(p + kNonceLen + ct_len, p + in.size());
  if (EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_GCM_SET_TAG, kTagLen, tag.data()) != 1 ||
      EVP_DecryptFinal_ex(ctx, o + len, &fin) != 1)
    throw std::invalid_argument("failed to decrypt: cipher: message authentication failed");
  return out;
}

}  // namespace pk_aes
