"""TensorBoard task (reference: ``harness/determined/exec/tensorboard.py``, which downloads the
event files of the chosen experiments/trials from checkpoint storage and runs TensorBoard).

TensorBoard/TensorFlow are not part of this image, so the task serves the scalar summaries
itself: it reads the TFRecord event files our trials write (``determined_amd.tensorboard``) from
``<storage>/tensorboard/experiment/<id>/trial/<id>/`` and exposes

* ``GET /data/runs``                           -> ``["exp-1/trial-2", ...]``
* ``GET /data/plugin/scalars/tags``            -> ``{run: {tag: {...}}}``
* ``GET /data/plugin/scalars/scalars?run=&tag=`` -> ``[[wall_time, step, value], ...]``
  (the same paths and shapes TensorBoard's scalar plugin uses), and
* ``GET /`` a self-contained HTML page plotting every tag (inline SVG, no external assets).

Event files are re-scanned on every request, so live trials show up as they report.

    python -m determined_amd.exec.tensorboard [--port P] (--experiment-ids 1,2 | --trial-ids 3 | LOGDIR...)
"""

import argparse
import html
import json
import os
import pathlib
import struct
import sys
import urllib.parse
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Any, Dict, List, Optional, Tuple

from determined_amd.tensorboard import decode_records


def _varint(buf: bytes, i: int) -> Tuple[int, int]:
    shift = n = 0
    while True:
        b = buf[i]
        i += 1
        n |= (b & 0x7F) << shift
        if not b & 0x80:
            return n, i
        shift += 7


def _fields(buf: bytes):
    """Iterate (field number, wire type, value) of a protobuf message."""
    i = 0
    while i < len(buf):
        key, i = _varint(buf, i)
        num, wire = key >> 3, key & 7
        if wire == 0:
            v, i = _varint(buf, i)
        elif wire == 1:
            v = buf[i : i + 8]
            i += 8
        elif wire == 2:
            ln, i = _varint(buf, i)
            v = buf[i : i + ln]
            i += ln
        elif wire == 5:
            v = buf[i : i + 4]
            i += 4
        else:
            raise ValueError(f"unsupported wire type {wire}")
        yield num, wire, v


def parse_scalar_events(path: str) -> List[Tuple[str, float, int, float]]:
    """``[(tag, wall_time, step, value)]`` from one event file (non-scalar records skipped)."""
    out = []
    for rec in decode_records(path):
        wall, step, summary = 0.0, 0, None
        for num, wire, v in _fields(rec):
            if num == 1 and wire == 1:
                wall = struct.unpack("<d", v)[0]
            elif num == 2 and wire == 0:
                step = v
            elif num == 5 and wire == 2:
                summary = v
        if summary is None:
            continue
        for num, wire, val in _fields(summary):
            if num != 1 or wire != 2:
                continue
            tag, value = None, None
            for n2, w2, x in _fields(val):
                if n2 == 1 and w2 == 2:
                    tag = x.decode()
                elif n2 == 2 and w2 == 5:
                    value = struct.unpack("<f", x)[0]
            if tag is not None and value is not None:
                out.append((tag, wall, step, value))
    return out


class ScalarStore:
    """Maps run names to directories and reads their event files on demand."""

    def __init__(self, runs: Dict[str, pathlib.Path]) -> None:
        self.runs = runs

    def scan(self) -> Dict[str, Dict[str, List[List[float]]]]:
        data: Dict[str, Dict[str, List[List[float]]]] = {}
        for run, root in self.runs.items():
            if not root.exists():
                continue
            for f in sorted(root.rglob("events.out.tfevents.*")):
                sub = f.parent.relative_to(root)
                name = run if str(sub) == "." else f"{run}/{sub}"
                for tag, wall, step, value in parse_scalar_events(str(f)):
                    data.setdefault(name, {}).setdefault(tag, []).append([wall, step, value])
        for tags in data.values():
            for pts in tags.values():
                pts.sort(key=lambda p: p[1])
        return data


PAGE = """<!doctype html><html><head><meta charset="utf-8"><title>determined_amd scalars</title>
<style>body{font-family:sans-serif;margin:16px}.c{display:inline-block;margin:8px;border:1px solid #ccc}
h3{font-size:13px;margin:4px}</style></head><body><h2>Scalars</h2><div id="g"></div><script>
const COLORS=["#1f77b4","#ff7f0e","#2ca02c","#d62728","#9467bd","#8c564b"];
fetch("data/plugin/scalars/all").then(r=>r.json()).then(d=>{const tags={};
for(const run in d)for(const t in d[run])(tags[t]=tags[t]||[]).push([run,d[run][t]]);
for(const t of Object.keys(tags).sort()){const W=420,H=240,P=36;let xs=[],ys=[];
for(const [r,pts] of tags[t])for(const p of pts){xs.push(p[1]);ys.push(p[2]);}
const x0=Math.min(...xs),x1=Math.max(...xs)||1,y0=Math.min(...ys),y1=Math.max(...ys);
const sx=v=>P+(W-2*P)*(x1>x0?(v-x0)/(x1-x0):0.5),sy=v=>H-P-(H-2*P)*(y1>y0?(v-y0)/(y1-y0):0.5);
let s=`<svg width=${W} height=${H}><text x=${P} y=14 font-size=11>${y1.toPrecision(4)}</text>`+
`<text x=${P} y=${H-P+24} font-size=11>${y0.toPrecision(4)} @ step ${x0}..${x1}</text>`;
tags[t].forEach(([r,pts],i)=>{s+=`<polyline fill=none stroke=${COLORS[i%6]} points="${
pts.map(p=>sx(p[1])+","+sy(p[2])).join(" ")}"><title>${r}</title></polyline>`;});
document.getElementById("g").insertAdjacentHTML("beforeend",`<div class=c><h3>${t}</h3>${s}</svg></div>`);}});
</script></body></html>"""


def make_handler(store: ScalarStore):
    class Handler(BaseHTTPRequestHandler):
        def log_message(self, *_: Any) -> None:
            pass

        def _send(self, code: int, body: bytes, ctype: str) -> None:
            self.send_response(code)
            self.send_header("Content-Type", ctype)
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

        def do_GET(self) -> None:
            u = urllib.parse.urlparse(self.path)
            q = {k: v[-1] for k, v in urllib.parse.parse_qs(u.query).items()}
            path = u.path.rstrip("/") or "/"
            # proxied paths keep a prefix (/proxy/<task>/...): match on the suffix
            for suffix in ("/data/runs", "/data/plugin/scalars/tags", "/data/plugin/scalars/scalars",
                           "/data/plugin/scalars/all"):
                if path.endswith(suffix):
                    data = store.scan()
                    if suffix == "/data/runs":
                        out: Any = sorted(data)
                    elif suffix.endswith("/tags"):
                        out = {r: {t: {"displayName": t} for t in tags} for r, tags in data.items()}
                    elif suffix.endswith("/all"):
                        out = data
                    else:
                        out = data.get(q.get("run", ""), {}).get(q.get("tag", ""), [])
                    return self._send(200, json.dumps(out).encode(), "application/json")
            if path == "/" or path.endswith("/index.html") or not os.path.splitext(path)[1]:
                return self._send(200, PAGE.encode(), "text/html")
            self._send(404, html.escape(path).encode(), "text/plain")

    return Handler


def resolve_runs(master: Optional[str], token: Optional[str], exp_ids: List[int], trial_ids: List[int],
                 logdirs: List[str]) -> Dict[str, pathlib.Path]:
    runs: Dict[str, pathlib.Path] = {f"logdir-{i}": pathlib.Path(d) for i, d in enumerate(logdirs)}
    if not (exp_ids or trial_ids):
        return runs
    from determined_amd.common.api import Session

    s = Session(master or os.environ["DET_MASTER"], token=token)

    def base_of(eid: int) -> pathlib.Path:
        cfg = s.get(f"/api/v1/experiments/{eid}")["config"]
        st = cfg.get("tensorboard_storage") or cfg["checkpoint_storage"]
        from determined_amd import storage

        sm = storage.build(st)
        rel = f"tensorboard/experiment/{eid}"
        if not getattr(sm, "is_local", True):  # object store: fetch the event files once
            import tempfile

            local = pathlib.Path(tempfile.mkdtemp(prefix=f"tb-exp-{eid}-"))
            try:
                sm.download(rel, local)
            except FileNotFoundError:
                pass
            return local
        return pathlib.Path(sm._base_path) / rel

    for eid in exp_ids:
        runs[f"exp-{eid}"] = base_of(eid)
    for tid in trial_ids:
        eid = s.get(f"/api/v1/trials/{tid}")["trial"]["experiment_id"]
        runs[f"exp-{eid}/trial-{tid}"] = base_of(eid) / "trial" / str(tid)
    return runs


def register_address(port: int) -> None:
    """Tell the master where this task listens (its proxy address)."""
    master, task = os.environ.get("DET_MASTER"), os.environ.get("DET_TASK_ID")
    if not (master and task):
        return
    from determined_amd.common.api import Session

    host = os.environ.get("DET_AGENT_HOST", "127.0.0.1")
    Session(master, token=os.environ.get("DET_SESSION_TOKEN") or None).post(
        f"/api/v1/tasks/{task}/proxy", {"host": host, "port": port})


def _ids(s: str) -> List[int]:
    return [int(x) for x in s.split(",") if x.strip()] if s else []


def main(argv: List[str]) -> int:
    ap = argparse.ArgumentParser(prog="tensorboard")
    ap.add_argument("--port", type=int, default=0)
    ap.add_argument("--host", default="127.0.0.1", help="bind address (read-only scalar viewer)")
    ap.add_argument("--experiment-ids", default="")
    ap.add_argument("--trial-ids", default="")
    ap.add_argument("logdirs", nargs="*")
    a = ap.parse_args(argv)
    runs = resolve_runs(os.environ.get("DET_MASTER"), os.environ.get("DET_SESSION_TOKEN") or None,
                        _ids(a.experiment_ids), _ids(a.trial_ids), a.logdirs)
    srv = ThreadingHTTPServer((a.host, a.port), make_handler(ScalarStore(runs)))
    srv.daemon_threads = True
    port = srv.server_address[1]
    print(f"tensorboard (scalars) serving {sorted(runs)} on port {port}", flush=True)
    register_address(port)
    try:
        srv.serve_forever()
    except KeyboardInterrupt:
        pass
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
