// AES-256-GCM secret cipher over OpenSSL 3 EVP, exposed to Python with pybind11.
//
// Behavioural contract = reference internal/adapters/security/cipher.go:
//   * key must be exactly 32 bytes (validateKey, cipher.go:15-23)
//   * Encrypt: fresh random 12-byte nonce; output = nonce || ciphertext || 16-byte tag,
//     no additional data (encryptKey, cipher.go:34-56)
//   * Decrypt: split the nonce off, error on short input or authentication failure
//     (decryptKey, cipher.go:61-83)
//   * BatchEncrypt/BatchDecrypt validate the key once and fail fast on the first error
//     (cipher.go:110-141)
// Error strings follow the Go messages so callers can match on them.
// The batch paths run with the GIL released and reuse one EVP context.
#include <openssl/evp.h>
#include <openssl/rand.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace py = pybind11;

namespace {

constexpr int kKeyLen = 32;
constexpr int kNonceLen = 12;
constexpr int kTagLen = 16;

struct CtxDeleter {
  void operator()(EVP_CIPHER_CTX* c) const { EVP_CIPHER_CTX_free(c); }
};
using CtxPtr = std::unique_ptr<EVP_CIPHER_CTX, CtxDeleter>;

void validate_key(const std::string& key) {
  if (key.size() != kKeyLen)
    throw std::invalid_argument("key length must be 32 bytes, got " + std::to_string(key.size()) + " bytes");
}

CtxPtr new_ctx() {
  CtxPtr c(EVP_CIPHER_CTX_new());
  if (!c) throw std::runtime_error("failed to create AES cipher: EVP_CIPHER_CTX_new");
  return c;
}

std::string seal(EVP_CIPHER_CTX* ctx, const std::string& key, const std::string& pt) {
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

std::string open(EVP_CIPHER_CTX* ctx, const std::string& key, const std::string& in) {
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

py::bytes encrypt(const std::string& key, const std::string& pt) {
  validate_key(key);
  std::string r;
  {
    py::gil_scoped_release nogil;
    auto c = new_ctx();
    r = seal(c.get(), key, pt);
  }
  return py::bytes(r);
}

py::bytes decrypt(const std::string& key, const std::string& data) {
  validate_key(key);
  std::string r;
  {
    py::gil_scoped_release nogil;
    auto c = new_ctx();
    r = open(c.get(), key, data);
  }
  return py::bytes(r);
}

template <bool kEncrypt>
py::list batch(const std::string& key, const std::vector<std::string>& items) {
  validate_key(key);
  std::vector<std::string> res;
  res.reserve(items.size());
  std::string err;
  bool bad_arg = false;
  {
    py::gil_scoped_release nogil;
    auto c = new_ctx();
    for (const auto& it : items) {
      try {
        res.push_back(kEncrypt ? seal(c.get(), key, it) : open(c.get(), key, it));
      } catch (const std::invalid_argument& e) {
        err = e.what();
        bad_arg = true;
        break;
      } catch (const std::exception& e) {
        err = e.what();
        break;
      }
    }
  }
  if (!err.empty()) {
    std::string msg = std::string(kEncrypt ? "failed to encrypt plaintext: " : "failed to decrypt ciphertext: ") + err;
    if (bad_arg) throw std::invalid_argument(msg);
    throw std::runtime_error(msg);
  }
  py::list out;
  for (auto& r : res) out.append(py::bytes(r));
  return out;
}

}  // namespace

PYBIND11_MODULE(_pk_aesgcm, m) {
  m.doc() = "AES-256-GCM (nonce||ct||tag) over OpenSSL EVP";
  m.attr("KEY_SIZE") = kKeyLen;
  m.attr("NONCE_SIZE") = kNonceLen;
  m.attr("TAG_SIZE") = kTagLen;
  m.def("validate_key", [](const std::string& k) { validate_key(k); });
  m.def("encrypt", &encrypt, py::arg("key"), py::arg("plaintext"));
  m.def("decrypt", &decrypt, py::arg("key"), py::arg("ciphertext"));
  m.def("batch_encrypt", &batch<true>, py::arg("key"), py::arg("plaintexts"));
  m.def("batch_decrypt", &batch<false>, py::arg("key"), py::arg("ciphertexts"));
}
