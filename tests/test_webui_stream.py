"""Master web UI page and the entity event stream it follows (reference: ``webui/react``,
``master/internal/stream``)."""

import threading
import time
import urllib.request

import pytest


@pytest.fixture()
def master():
    from determined_amd.common.api import Session
    from determined_amd.master import start_master

    srv = start_master()
    yield srv, Session(f"http://127.0.0.1:{srv.port}")
    srv.stop()


def test_webui_page_is_served(master):
    srv, _ = master
    for path in ("/", "/det/"):
        with urllib.request.urlopen(f"http://127.0.0.1:{srv.port}{path}", timeout=10) as r:
            assert r.headers["Content-Type"].startswith("text/html")
            body = r.read().decode()
        assert "determined-amd" in body and "/ui/app.js" in body and "#/runs" in body and "#/jobs" in body
    with urllib.request.urlopen(f"http://127.0.0.1:{srv.port}/ui/app.js", timeout=10) as r:
        assert r.headers["Content-Type"].startswith("application/javascript")
        js = r.read().decode()
    assert "/api/v1/stream" in js and "/api/v1/runs" in js and "parallel(" in js
    with urllib.request.urlopen(f"http://127.0.0.1:{srv.port}/ui/app.css", timeout=10) as r:
        assert r.headers["Content-Type"].startswith("text/css")


def test_stream_long_poll_delivers_entity_changes(master):
    srv, s = master
    cfg = {"name": "stream", "entrypoint": "model_def:T", "hyperparameters": {},
           "searcher": {"name": "single", "metric": "loss", "max_length": {"batches": 1}}}
    first = s.get("/api/v1/stream", params={"since": 0})
    seq = first["last_seq"]
    got = {}

    def poll():
        got["r"] = s.get("/api/v1/stream", params={"since": seq, "timeout_seconds": 20, "entities": "experiment"},
                         timeout=30)

    t = threading.Thread(target=poll)
    t.start()
    time.sleep(0.3)  # the poll is parked before the change happens
    eid = s.post("/api/v1/experiments", {"config": cfg, "activate": False})["experiment"]["id"]
    t.join(30)
    evs = got["r"]["events"]
    assert evs and all(e["entity"] == "experiment" for e in evs) and any(e["id"] == eid for e in evs)
    assert all("config" not in e["fields"] and "model_def" not in e["fields"] for e in evs)
    s.post(f"/api/v1/experiments/{eid}/archive", {})
    nxt = s.get("/api/v1/stream", params={"since": got["r"]["last_seq"], "entities": "experiment"})
    assert any(e["fields"].get("archived") in (1, True) for e in nxt["events"])
    # a cursor older than the ring asks the client to resync
    m = srv.master
    for i in range(m.stream_events.maxlen + 5):
        m.db.update("tasks", "id", "nope", state="X")
    assert s.get("/api/v1/stream", params={"since": 1})["resync"] is True
    # a cursor from an earlier master process: ahead of this sequence, or another epoch
    cur = s.get("/api/v1/stream", params={"since": m.stream_seq})
    assert cur["resync"] is False and cur["epoch"] == m.stream_epoch
    assert s.get("/api/v1/stream", params={"since": m.stream_seq + 100})["resync"] is True
    assert s.get("/api/v1/stream", params={"since": m.stream_seq, "epoch": "old-process"})["resync"] is True
    assert s.get("/api/v1/stream", params={"since": m.stream_seq, "epoch": cur["epoch"]})["resync"] is False


@pytest.mark.skipif(__import__("shutil").which("node") is None, reason="node not installed")
def test_webui_script_renders_every_view_against_a_live_master(master, tmp_path):
    """Run the app's script under node with a minimal DOM stub: every view (and every experiment
    tab) renders from the real API responses without a script error."""
    import json
    import subprocess

    from determined_amd.master._webui import ASSETS

    srv, s = master
    cfg = {"name": "ui", "entrypoint": "model_def:T", "hyperparameters": {"lr": {"type": "double", "minval": 0.001,
                                                                                  "maxval": 0.1}, "opt": "sgd"},
           "searcher": {"name": "random", "metric": "loss", "max_trials": 3, "max_length": {"batches": 1}}}
    eid = s.post("/api/v1/experiments", {"config": cfg})["experiment"]["id"]
    trials = s.get(f"/api/v1/experiments/{eid}/trials")["trials"]
    assert trials
    tid = trials[0]["id"]
    base = f"http://127.0.0.1:{srv.port}"
    views = ["#/experiments"] + [f"#/experiments/{eid}/{t}" for t in
                                 ("overview", "trials", "hp", "compare", "checkpoints", "config", "code")] + \
        [f"#/trials/{tid}", "#/runs", "#/projects", "#/projects/1", "#/jobs", "#/cluster", "#/tasks", "#/models",
         "#/admin"]
    harness = """
const els = {};
function el(id) { return els[id] || (els[id] = {innerHTML: "", textContent: "", scrollTop: 0, scrollHeight: 0,
  classList: {add() {}, remove() {}, toggle() {}}, addEventListener() {}, onclick: null}); }
global.document = {querySelector: s => el(s), querySelectorAll: () => []};
global.localStorage = {getItem: () => "", setItem() {}};
global.window = {DAMD_TEST: true};
const http = require("http");
global.fetch = (p, o) => new Promise((resolve, reject) => {  // node 12 has no fetch: a minimal one
  o = o || {};
  const req = http.request(BASE + p, {method: o.method || "GET", headers: o.headers || {}}, res => {
    let body = "";
    res.on("data", c => body += c);
    res.on("end", () => resolve({status: res.statusCode, ok: res.statusCode < 300, json: async () => JSON.parse(body)}));
  });
  req.on("error", reject);
  if (o.body) req.write(o.body);
  req.end();
});
global.location = {hash: "#/"};
const app = require(APP);
(async () => {
  for (const h of VIEWS) {
    location.hash = h; await app.route();
    if (els["#err"].textContent) { console.log("ERR " + h + " " + els["#err"].textContent); process.exit(1); }
    console.log("OK " + h + " " + els["#view"].innerHTML.length);
  }
})();
""".replace("BASE", json.dumps(base)).replace("APP", json.dumps(str(ASSETS / "app.js"))).replace(
        "VIEWS", json.dumps(views))
    f = tmp_path / "ui_test.js"
    f.write_text(harness)
    out = subprocess.run(["node", str(f)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    ok = [ln for ln in out.stdout.splitlines() if ln.startswith("OK ")]
    assert len(ok) == len(views), out.stdout
    assert all(int(ln.split()[-1]) > 100 for ln in ok), out.stdout  # every view rendered content
