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

#include "security/aes_gcm_core.h"

namespace {
using namespace pk_aes;

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
