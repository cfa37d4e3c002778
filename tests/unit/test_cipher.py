"""AES-256-GCM C++ extension vs reference cipher.go semantics."""
import base64
import json

import pytest

from polykey_service_amd.adapters.security import SecretStore, cipher, parse_key

KEY = bytes(range(32))


def test_roundtrip_and_layout():
    for pt in (b"", b"x", b"hello world" * 100):
        ct = cipher.encrypt(KEY, pt)
        assert len(ct) == 12 + len(pt) + 16
        assert cipher.decrypt(KEY, ct) == pt


def test_nonce_is_random():
    a, b = cipher.encrypt(KEY, b"same"), cipher.encrypt(KEY, b"same")
    assert a[:12] != b[:12] and a != b


@pytest.mark.parametrize("n", [0, 16, 31, 33, 64])
def test_key_length(n):
    with pytest.raises(ValueError, match=f"key length must be 32 bytes, got {n} bytes"):
        cipher.encrypt(bytes(n), b"x")
    with pytest.raises(ValueError, match="key length"):
        cipher.decrypt(bytes(n), b"x" * 40)


def test_short_and_tampered():
    with pytest.raises(ValueError, match="ciphertext too short: 11 bytes, expected at least 12 bytes"):
        cipher.decrypt(KEY, b"a" * 11)
    ct = bytearray(cipher.encrypt(KEY, b"secret"))
    for i in (0, 12, len(ct) - 1):
        bad = bytearray(ct)
        bad[i] ^= 0x80
        with pytest.raises(ValueError, match="message authentication failed"):
            cipher.decrypt(KEY, bytes(bad))
    with pytest.raises(ValueError, match="authentication failed"):
        cipher.decrypt(bytes(reversed(KEY)), bytes(ct))


def test_batch_fail_fast():
    cts = cipher.batch_encrypt(KEY, [b"a", b"b", b"c"])
    assert cipher.batch_decrypt(KEY, cts) == [b"a", b"b", b"c"]
    with pytest.raises(ValueError, match="^failed to decrypt ciphertext: "):
        cipher.batch_decrypt(KEY, [cts[0], b"short", cts[2]])
    with pytest.raises(ValueError, match="key length"):
        cipher.batch_encrypt(b"k", [b"a"])
    assert cipher.batch_encrypt(KEY, []) == []


def test_secret_store_from_env(tmp_path):
    blob = cipher.encrypt(KEY, b"provider")
    p = tmp_path / "s.json"
    p.write_text(json.dumps({"sid": base64.b64encode(blob).decode()}))
    st = SecretStore.from_env({"POLYKEY_MASTER_KEY": KEY.hex(), "POLYKEY_SECRETS_FILE": str(p)})
    assert st.get("sid") == b"provider" and st.get("nope") is None
    assert parse_key(base64.b64encode(KEY).decode()) == KEY
    assert SecretStore.from_env({}) is None
