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


class _CookieSvc(_Svc):
    seen = []

    def do_GET(self):
        _CookieSvc.seen.append(self.headers.get("Cookie"))
        super().do_GET()


def test_proxy_requires_access_to_the_task_and_never_forwards_the_session(tmp_path):
    """another user can neither reach nor retarget someone else's task service,
    registration is the task's own (cluster token) and bounded to loopback / agent hosts, and the
    master's ``auth`` session cookie is stripped before forwarding."""
    from determined_amd.master import start_master

    port = free_port()
    srv = http.server.ThreadingHTTPServer(("127.0.0.1", port), _CookieSvc)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    m = start_master(auth="basic", auth_token="cluster-secret")
    try:
        url = f"http://127.0.0.1:{m.port}"

        def login(user, pw=""):
            return Session(url, token=Session(url).post("/api/v1/auth/login",
                                                        {"username": user, "password": pw})["token"])

        admin = login("admin")
        admin.post("/api/v1/users", {"username": "alice", "password": "a"})
        admin.post("/api/v1/users", {"username": "bob", "password": "b"})
        alice, bob = login("alice", "a"), login("bob", "b")
        tid = alice.post("/api/v1/commands", {"command": ["sleep", "1"], "slots": 0, "type": "TENSORBOARD"})["task_id"]
        task = Session(url, token="cluster-secret")
        # only the task itself (cluster token) or an admin registers; never an arbitrary host
        with pytest.raises(Exception, match="403"):
            bob.post(f"/api/v1/tasks/{tid}/proxy", {"host": "127.0.0.1", "port": port})
        with pytest.raises(Exception, match="400"):
            task.post(f"/api/v1/tasks/{tid}/proxy", {"host": "evil.example.com", "port": port})
        task.post(f"/api/v1/tasks/{tid}/proxy", {"host": "127.0.0.1", "port": port})
        # the owner reaches it (token in the cookie, as a browser would); the auth cookie is stripped
        r = requests.get(f"{url}/proxy/{tid}/x", cookies={"auth": alice.token, "theme": "dark"})
        assert r.status_code == 200 and r.text == "svc saw /x"
        assert _CookieSvc.seen[-1] == "theme=dark"
        # another non-admin user gets a 404 and the upstream never sees the request
        n = len(_CookieSvc.seen)
        r = requests.get(f"{url}/proxy/{tid}/x", cookies={"auth": bob.token})
        assert r.status_code == 404
        r = requests.get(f"{url}/proxy/{tid}/x", headers={"Authorization": f"Bearer {bob.token}"})
        assert r.status_code == 404
        assert len(_CookieSvc.seen) == n
        # an admin may
        assert requests.get(f"{url}/proxy/{tid}/y", headers={"Authorization": f"Bearer {admin.token}"}).status_code == 200
        # unauthenticated: 401
        assert requests.get(f"{url}/proxy/{tid}/x").status_code == 401
    finally:
        srv.shutdown()
        m.stop()
        m.master.close()
