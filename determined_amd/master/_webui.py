"""Web UI served by the master at ``/`` (reference: ``webui/react``, a React app over the REST API).

One self-contained page (no build step, no external assets -- the cluster may have no egress):
experiment list with state / progress / actions, experiment detail with its trials and their
searcher-metric curves (inline SVG), trial detail with training / validation curves, checkpoints
and live logs, cluster view (agents, slots, resource pools, job queue, NTSC tasks) and the model
registry.  Everything is fetched from ``/api/v1``; the page long-polls ``/api/v1/stream`` and
re-renders the current view when an entity it shows changes.  With authentication enabled the
page asks for credentials and keeps the session token in ``localStorage``.
"""

PAGE = r"""<!doctype html>
<html><head><meta charset="utf-8"><title>determined-amd</title>
<style>
body{font-family:system-ui,sans-serif;margin:0;background:#f6f7f9;color:#1d232b}
header{background:#1d232b;color:#fff;padding:10px 18px;display:flex;gap:18px;align-items:center}
header a{color:#cfd8e3;text-decoration:none}header a.on{color:#fff;font-weight:600}
main{padding:16px 18px}table{border-collapse:collapse;width:100%;background:#fff}
th,td{padding:6px 8px;border-bottom:1px solid #e4e7eb;text-align:left;font-size:13px;vertical-align:top}
th{background:#eef1f4}.st{padding:2px 6px;border-radius:8px;font-size:11px;color:#fff;background:#7b8794}
.ACTIVE,.RUNNING{background:#2f80ed}.COMPLETED,.TERMINATED{background:#27ae60}.ERROR{background:#eb5757}
.CANCELED,.PAUSED{background:#f2994a}.bar{height:6px;background:#e4e7eb;width:90px}.bar>div{height:6px;background:#2f80ed}
button{font-size:12px;margin-right:4px}pre{background:#0f1419;color:#d6deeb;padding:8px;max-height:360px;overflow:auto;font-size:12px}
.card{background:#fff;padding:12px;margin-bottom:14px;border:1px solid #e4e7eb}h2{font-size:16px;margin:4px 0 10px}
#err{color:#eb5757}svg text{font-size:10px;fill:#52606d}
</style></head><body>
<header><b>determined-amd</b><a href="#/" id="n-exp">Experiments</a><a href="#/cluster" id="n-cluster">Cluster</a>
<a href="#/models" id="n-models">Models</a><span id="who" style="margin-left:auto"></span></header>
<main><div id="err"></div><div id="view">loading...</div></main>
<script>
const $ = s => document.querySelector(s);
let token = localStorage.getItem("det_token") || "";
let seq = 0, epoch = "";
async function api(path, opts = {}) {
  const h = {"Content-Type": "application/json"};
  if (token) h["Authorization"] = "Bearer " + token;
  const r = await fetch(path, Object.assign({headers: h}, opts));
  if (r.status === 401) { showLogin(); throw new Error("login required"); }
  const j = await r.json();
  if (!r.ok) throw new Error(j.error || r.status);
  return j;
}
function esc(v) { return String(v === undefined || v === null ? "" : v).replace(/[&<>"]/g, c => ({"&":"&amp;","<":"&lt;",">":"&gt;","\"":"&quot;"})[c]); }
function st(s) { return `<span class="st ${esc(s)}">${esc(s)}</span>`; }
function ts(t) { return t ? new Date(t * 1000).toLocaleString() : ""; }
function showLogin() {
  $("#view").innerHTML = `<div class="card"><h2>Sign in</h2><input id="u" placeholder="user" value="determined">
   <input id="p" type="password" placeholder="password"><button id="go">Sign in</button></div>`;
  $("#go").onclick = async () => {
    const r = await fetch("/api/v1/auth/login", {method: "POST", body: JSON.stringify({username: $("#u").value, password: $("#p").value})});
    const j = await r.json();
    if (!r.ok) { $("#err").textContent = j.error || "login failed"; return; }
    token = j.token; localStorage.setItem("det_token", token); route();
  };
}
function chart(series, w = 560, h = 200) {
  // series: [{name, pts: [[x, y], ...]}]
  const all = series.flatMap(s => s.pts);
  if (!all.length) return "<i>no metrics yet</i>";
  const xs = all.map(p => p[0]), ys = all.map(p => p[1]);
  const x0 = Math.min(...xs), x1 = Math.max(...xs) || 1, y0 = Math.min(...ys), y1 = Math.max(...ys);
  const sx = x => 40 + (w - 50) * (x1 === x0 ? 0.5 : (x - x0) / (x1 - x0));
  const sy = y => h - 20 - (h - 30) * (y1 === y0 ? 0.5 : (y - y0) / (y1 - y0));
  const col = ["#2f80ed","#eb5757","#27ae60","#f2994a","#9b51e0","#56ccf2","#219653","#bb6bd9"];
  let out = `<svg width="${w}" height="${h}"><line x1="40" y1="${h-20}" x2="${w-10}" y2="${h-20}" stroke="#aaa"/>
    <line x1="40" y1="10" x2="40" y2="${h-20}" stroke="#aaa"/><text x="2" y="14">${y1.toPrecision(4)}</text>
    <text x="2" y="${h-22}">${y0.toPrecision(4)}</text><text x="40" y="${h-6}">${x0}</text><text x="${w-60}" y="${h-6}">${x1}</text>`;
  series.forEach((s, i) => {
    const p = s.pts.map(q => `${sx(q[0]).toFixed(1)},${sy(q[1]).toFixed(1)}`).join(" ");
    out += `<polyline fill="none" stroke="${col[i % col.length]}" stroke-width="1.5" points="${p}"/>
      <text x="${w - 150}" y="${14 + 12 * i}" style="fill:${col[i % col.length]}">${esc(s.name)}</text>`;
  });
  return out + "</svg>";
}
async function act(kind, id, a) { try { await api(`/api/v1/${kind}/${id}/${a}`, {method: "POST", body: "{}"}); route(); } catch (e) { $("#err").textContent = e; } }
async function viewExperiments() {
  const d = await api("/api/v1/experiments");
  const rows = d.experiments.map(e => `<tr><td><a href="#/exp/${e.id}">${e.id}</a></td><td>${esc(e.name)}</td><td>${st(e.state)}</td>
    <td><div class="bar"><div style="width:${Math.round(100 * (e.progress || 0))}%"></div></div></td><td>${esc(e.searcher_type)}</td>
    <td>${e.num_trials}</td><td>${esc((e.labels || []).join(", "))}</td><td>${ts(e.start_time)}</td><td>
    <button onclick="act('experiments',${e.id},'pause')">pause</button><button onclick="act('experiments',${e.id},'activate')">activate</button>
    <button onclick="act('experiments',${e.id},'kill')">kill</button><button onclick="act('experiments',${e.id},'archive')">archive</button></td></tr>`).join("");
  return `<div class="card"><h2>Experiments</h2><table><tr><th>ID</th><th>Name</th><th>State</th><th>Progress</th><th>Searcher</th>
    <th>Trials</th><th>Labels</th><th>Started</th><th></th></tr>${rows}</table></div>`;
}
async function curves(trials, group, metric) {
  const out = [];
  for (const t of trials.slice(0, 16)) {
    const m = await api(`/api/v1/trials/${t.id}/metrics?group=${group}`);
    const pts = m.metrics.filter(r => r.metrics && r.metrics[metric] !== undefined).map(r => [r.steps_completed, r.metrics[metric]]);
    if (pts.length) out.push({name: `trial ${t.id}`, pts});
  }
  return out;
}
async function viewExperiment(id) {
  const e = await api(`/api/v1/experiments/${id}`);
  const tr = (await api(`/api/v1/experiments/${id}/trials`)).trials;
  const metric = ((e.config || {}).searcher || {}).metric;
  const rows = tr.map(t => `<tr><td><a href="#/trial/${t.id}">${t.id}</a></td><td>${st(t.state)}</td><td>${esc(JSON.stringify(t.hparams))}</td>
    <td>${esc(t.best_validation)}</td><td>${t.total_batches}</td><td>${t.restarts}</td><td>${esc(t.latest_checkpoint)}</td></tr>`).join("");
  const ck = (await api(`/api/v1/experiments/${id}/checkpoints`)).checkpoints || [];
  const ckr = ck.slice(-20).map(c => `<tr><td>${esc(c.uuid)}</td><td>${c.trial_id}</td><td>${c.steps_completed}</td><td>${st(c.state)}</td></tr>`).join("");
  return `<div class="card"><h2>Experiment ${id}: ${esc((e.experiment || e).name || "")} ${st((e.experiment || e).state)}</h2>
    <div>validation <b>${esc(metric)}</b></div>${chart(await curves(tr, "validation", metric))}</div>
    <div class="card"><h2>Trials</h2><table><tr><th>ID</th><th>State</th><th>Hyperparameters</th><th>Best validation</th><th>Batches</th>
    <th>Restarts</th><th>Latest checkpoint</th></tr>${rows}</table></div>
    <div class="card"><h2>Checkpoints</h2><table><tr><th>UUID</th><th>Trial</th><th>Steps</th><th>State</th></tr>${ckr}</table></div>
    <div class="card"><h2>Configuration</h2><pre>${esc(JSON.stringify(e.config, null, 2))}</pre></div>`;
}
async function viewTrial(id) {
  const t = (await api(`/api/v1/trials/${id}`)).trial;
  const m = (await api(`/api/v1/trials/${id}/metrics`)).metrics;
  const series = {};
  for (const r of m) for (const [k, v] of Object.entries(r.metrics || {})) if (typeof v === "number") {
    const n = `${r.group_name}/${k}`; (series[n] = series[n] || []).push([r.steps_completed, v]); }
  const logs = (await api(`/api/v1/tasks/trial-${id}/logs?limit=400`)).logs.slice(-400).map(l => esc(l.log)).join("\n");
  const ck = (await api(`/api/v1/trials/${id}/checkpoints`)).checkpoints || [];
  return `<div class="card"><h2>Trial ${id} ${st(t.state)} <button onclick="act('trials',${id},'kill')">kill</button></h2>
    <div>hyperparameters: <code>${esc(JSON.stringify(t.hparams))}</code> | batches ${t.total_batches} | restarts ${t.restarts}</div>
    ${chart(Object.entries(series).map(([name, pts]) => ({name, pts})))}</div>
    <div class="card"><h2>Checkpoints</h2>${ck.map(c => esc(c.uuid) + " @ " + c.steps_completed).join("<br>")}</div>
    <div class="card"><h2>Logs</h2><pre>${logs}</pre></div>`;
}
async function viewCluster() {
  const ag = (await api("/api/v1/agents")).agents, rp = (await api("/api/v1/resource-pools")).resource_pools;
  const jobs = (await api("/api/v1/job-queues")).jobs, tasks = (await api("/api/v1/tasks")).tasks;
  return `<div class="card"><h2>Resource pools</h2><table><tr><th>Name</th><th>Scheduler</th><th>Slots used / total</th><th>Agents</th></tr>
    ${rp.map(p => `<tr><td>${esc(p.name)}</td><td>${esc(p.scheduler_type)}</td><td>${p.slots_used} / ${p.slots_available}</td><td>${p.num_agents}</td></tr>`).join("")}</table></div>
    <div class="card"><h2>Agents</h2><table><tr><th>ID</th><th>Host</th><th>Slots</th><th>GPU</th><th>Enabled</th><th>Label</th></tr>
    ${ag.map(a => `<tr><td>${esc(a.id)}</td><td>${esc(a.host)}</td><td>${a.slots}</td><td>${a.gpu}</td><td>${a.enabled}</td><td>${esc(a.label)}</td></tr>`).join("")}</table></div>
    <div class="card"><h2>Job queue</h2><pre>${esc(JSON.stringify(jobs, null, 1))}</pre></div>
    <div class="card"><h2>Tasks</h2><table><tr><th>ID</th><th>Type</th><th>State</th><th>Started</th><th>Exit</th></tr>
    ${tasks.map(t => `<tr><td>${esc(t.id)}</td><td>${esc(t.type)}</td><td>${st(t.state)}</td><td>${ts(t.start_time)}</td><td>${esc(t.exit_code)}</td></tr>`).join("")}</table></div>`;
}
async function viewModels() {
  const ms = (await api("/api/v1/models")).models;
  return `<div class="card"><h2>Model registry</h2><table><tr><th>Name</th><th>Description</th><th>Labels</th><th>Created</th></tr>
    ${ms.map(m => `<tr><td>${esc(m.name)}</td><td>${esc(m.description)}</td><td>${esc((m.labels || []).join(", "))}</td><td>${ts(m.creation_time)}</td></tr>`).join("")}</table></div>`;
}
async function route() {
  const h = location.hash || "#/";
  document.querySelectorAll("header a").forEach(a => a.classList.remove("on"));
  $("#err").textContent = "";
  try {
    let html;
    if (h.startsWith("#/exp/")) html = await viewExperiment(+h.split("/")[2]);
    else if (h.startsWith("#/trial/")) html = await viewTrial(+h.split("/")[2]);
    else if (h === "#/cluster") { $("#n-cluster").classList.add("on"); html = await viewCluster(); }
    else if (h === "#/models") { $("#n-models").classList.add("on"); html = await viewModels(); }
    else { $("#n-exp").classList.add("on"); html = await viewExperiments(); }
    $("#view").innerHTML = html;
  } catch (e) { if (String(e).indexOf("login") < 0) $("#err").textContent = e; }
}
async function follow() {  // live updates: long-poll the master's event stream
  for (;;) {
    try {
      const d = await api(`/api/v1/stream?since=${seq}&timeout_seconds=25&epoch=${epoch}`);
      const changed = d.resync || d.events.length > 0;
      seq = d.last_seq; epoch = d.epoch || "";
      if (changed) await route();
    } catch (e) { await new Promise(r => setTimeout(r, 3000)); }
  }
}
window.onhashchange = route;
api("/api/v1/me").then(u => { $("#who").textContent = (u.user || {}).username || ""; }).catch(() => {});
route().then(follow);
</script></body></html>
"""


def add_webui_routes(route, _Raw) -> None:
    for path in ("/", "/det", "/det/", "/ui", "/ui/"):
        route("GET", path)(lambda q, b: _Raw(PAGE, "text/html; charset=utf-8"))
