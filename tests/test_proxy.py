"""The master's task proxy (reference master/internal/proxy): ``/proxy/<task_id>/...`` forwards to
the service a task registered (notebook / TensorBoard port)."""

import http.server
import threading

import pytest
import requests

from determined_amd.common.api import Session
from tests.dist_utils import free_port


class _Svc(http.server.BaseHTTPRequestHandler):
    def do_GET(self):
        body = f"svc saw {self.path}".encode()
        self.send_response(200)
        self.send_header("Content-Type", "text/plain")
        self.send_header("X-Svc", "1")
        self.send_header("Content-Length", str(len(body)))
        self.end_headers()
        self.wfile.write(body)

    def do_POST(self):
        n = int(self.headers.get("Content-Length") or 0)
        body = b"echo:" + self.rfile.read(n)
        self.send_response(201)
        self.send_header("Content-Length", str(len(body)))
        self.end_headers()
        self.wfile.write(body)

    def log_message(self, *a):
        pass


@pytest.fixture()
def svc():
    port = free_port()
    srv = http.server.ThreadingHTTPServer(("127.0.0.1", port), _Svc)
    t = threading.Thread(target=srv.serve_forever, daemon=True)
    t.start()
    yield port
    srv.shutdown()


def test_proxy_forwards_to_registered_task_service(svc):
    from determined_amd.master import start_master

    m = start_master()
    try:
        url = f"http://127.0.0.1:{m.port}"
        s = Session(url)
        tid = s.post("/api/v1/commands", {"command": ["sleep", "1"], "slots": 0, "type": "TENSORBOARD"})["task_id"]
        r = requests.get(f"{url}/proxy/{tid}/x")
        assert r.status_code == 404  # nothing registered yet
        s.post(f"/api/v1/tasks/{tid}/proxy", {"host": "127.0.0.1", "port": svc})
        r = requests.get(f"{url}/proxy/{tid}/data/scalars?run=a")
        assert r.status_code == 200 and r.text == "svc saw /data/scalars?run=a" and r.headers["X-Svc"] == "1"
        r = requests.post(f"{url}/proxy/{tid}/api", data=b"payload")
        assert r.status_code == 201 and r.content == b"echo:payload"
    finally:
        m.stop()
        m.master.close()
