"""Optional TLS transport (SURVEY.md §5.9 [NEW]): a server started with a PEM certificate and
key serves ExecuteTool over TLS; plaintext clients are refused; the dev client verifies the
server with ``POLYKEY_TLS_CA``.  The certificate is a throwaway self-signed one made by the
openssl CLI for 127.0.0.1."""
import io
import shutil
import subprocess

import grpc
import pytest

from polykey_service_amd import proto
from polykey_service_amd.client import dev_client
from polykey_service_amd.config.server_config import load_server_config
from tests.helpers import ServerThread

pytestmark = pytest.mark.skipif(shutil.which("openssl") is None, reason="openssl CLI not available")


@pytest.fixture(scope="module")
def cert(tmp_path_factory):
    d = tmp_path_factory.mktemp("tls")
    crt, key = d / "server.crt", d / "server.key"
    subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-days", "1", "-subj", "/CN=localhost",
                    "-addext", "subjectAltName=IP:127.0.0.1,DNS:localhost", "-keyout", str(key), "-out", str(crt)],
                   check=True, capture_output=True)
    return str(crt), str(key)


def test_tls_round_trip_and_plaintext_refused(cert):
    crt, key = cert
    with ServerThread(tls_cert=crt, tls_key=key) as s:
        with open(crt, "rb") as f:
            creds = grpc.ssl_channel_credentials(root_certificates=f.read())
        with grpc.secure_channel(s.addr, creds) as ch:
            call = ch.unary_unary(proto.EXECUTE_TOOL, request_serializer=proto.ExecuteToolRequest.SerializeToString,
                                  response_deserializer=proto.ExecuteToolResponse.FromString)
            r = call(dev_client.build_request("example_tool"), timeout=10)
            assert r.status.code == 200
        with grpc.insecure_channel(s.addr) as ch:
            call = ch.unary_unary(proto.EXECUTE_TOOL, request_serializer=proto.ExecuteToolRequest.SerializeToString,
                                  response_deserializer=proto.ExecuteToolResponse.FromString)
            with pytest.raises(grpc.RpcError):
                call(dev_client.build_request("example_tool"), timeout=3)
        starting = [r for r in s.records() if r["msg"] == "server starting"]
        assert starting and starting[0].get("tls") is True


def test_dev_client_over_tls(cert, monkeypatch):
    crt, key = cert
    with ServerThread(tls_cert=crt, tls_key=key) as s:
        monkeypatch.setenv("POLYKEY_SERVER_ADDR", s.addr)
        monkeypatch.setenv("POLYKEY_TLS_CA", crt)
        out = io.StringIO()
        assert dev_client.main([], out=out) == 0
    assert "All 4 checks passed" in out.getvalue()


def test_server_config_tls_fields():
    cfg = load_server_config(["--tls-cert", "/c.pem"], environ={"POLYKEY_TLS_KEY": "/k.pem"})
    assert cfg.tls_cert == "/c.pem" and cfg.tls_key == "/k.pem"
