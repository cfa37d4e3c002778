"""Secret store keyed by ``secret_id`` (the field of ``ExecuteToolRequest``, ``server.go:31``).

The reference carries ``secret_id`` through to the service but never resolves it and has an
AES-GCM cipher with no callers.  Here secrets are kept *encrypted at rest*
with the same cipher and decrypted only when a tool that declares ``requires_secret`` runs.

Sources: ``POLYKEY_MASTER_KEY`` (32 bytes as 64 hex chars or base64) and optionally
``POLYKEY_SECRETS_FILE`` — JSON ``{secret_id: base64(nonce||ct||tag)}``.
"""
from __future__ import annotations

import base64
import binascii
import json
import os
import threading
from typing import Dict, Mapping, Optional

from . import cipher


def parse_key(text: str) -> bytes:
    text = text.strip()
    try:
        k = binascii.unhexlify(text)
        if len(k) == cipher.KEY_SIZE:
            return k
    except (binascii.Error, ValueError):
        pass
    k = base64.b64decode(text)
    cipher.validate_key(k)
    return k


class SecretStore:
    def __init__(self, master_key: bytes):
        cipher.validate_key(master_key)
        self._key = master_key
        self._blobs: Dict[str, bytes] = {}
        self._lock = threading.Lock()

    @classmethod
    def from_env(cls, environ: Optional[Mapping[str, str]] = None) -> Optional["SecretStore"]:
        env = os.environ if environ is None else environ
        raw = env.get("POLYKEY_MASTER_KEY", "")
        if not raw:
            return None
        store = cls(parse_key(raw))
        path = env.get("POLYKEY_SECRETS_FILE", "")
        if path:
            with open(path) as f:
                for sid, b64 in json.load(f).items():
                    store.put_encrypted(sid, base64.b64decode(b64))
        return store

    def put(self, secret_id: str, plaintext: bytes) -> None:
        blob = cipher.encrypt(self._key, plaintext)
        with self._lock:
            self._blobs[secret_id] = blob

    def put_encrypted(self, secret_id: str, blob: bytes) -> None:
        with self._lock:
            self._blobs[secret_id] = bytes(blob)

    def get(self, secret_id: str) -> Optional[bytes]:
        with self._lock:
            blob = self._blobs.get(secret_id)
        if blob is None:
            return None
        return cipher.decrypt(self._key, blob)

    def export(self) -> Dict[str, str]:
        with self._lock:
            return {k: base64.b64encode(v).decode() for k, v in self._blobs.items()}

    def __contains__(self, secret_id: str) -> bool:
        return secret_id in self._blobs
