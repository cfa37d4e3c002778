"""AES-256-GCM secret cipher (reference ``internal/adapters/security/cipher.go``).

Thin Python face over the C++/OpenSSL extension ``_pk_aesgcm`` (``csrc/security/aes_gcm.cpp``).
Byte layout is identical to the reference: ``nonce(12) || ciphertext || tag(16)``, no AAD.
``ValueError`` carries the reference's error strings (``key length must be 32 bytes, got N
bytes``, ``ciphertext too short: ...``, ``failed to decrypt: cipher: message authentication
failed``; batch variants prefix ``failed to encrypt plaintext:`` / ``failed to decrypt
ciphertext:`` and fail fast, ``cipher.go:110-141``).
"""
from __future__ import annotations

from typing import List, Sequence

from ..._native.loader import load_extension

_ext = load_extension("_pk_aesgcm")

KEY_SIZE = _ext.KEY_SIZE
NONCE_SIZE = _ext.NONCE_SIZE
TAG_SIZE = _ext.TAG_SIZE


def validate_key(key: bytes) -> None:
    _ext.validate_key(bytes(key))


def encrypt(key: bytes, plaintext: bytes) -> bytes:
    return _ext.encrypt(bytes(key), bytes(plaintext))


def decrypt(key: bytes, ciphertext: bytes) -> bytes:
    return _ext.decrypt(bytes(key), bytes(ciphertext))


def batch_encrypt(key: bytes, plaintexts: Sequence[bytes]) -> List[bytes]:
    return _ext.batch_encrypt(bytes(key), [bytes(p) for p in plaintexts])


def batch_decrypt(key: bytes, ciphertexts: Sequence[bytes]) -> List[bytes]:
    return _ext.batch_decrypt(bytes(key), [bytes(c) for c in ciphertexts])
