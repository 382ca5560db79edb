// determined-amd web UI: a dependency-free single-page app over the master's REST API
// (reference: webui/react -- experiment list / detail with trial comparison and hyperparameter
// visualisation, flat runs, projects, job queue, cluster, tasks, model registry, admin).
// Hash routes: #/experiments, #/experiments/<id>/<tab>, #/trials/<id>, #/runs, #/projects[/<ws>],
// #/jobs, #/cluster, #/tasks[/<id>], #/models[/<name>], #/admin.  Live: the page long-polls
// /api/v1/stream and re-renders the current view when an entity changes.
"use strict";

const $ = s => document.querySelector(s);
const COLORS = ["#2f80ed", "#eb5757", "#27ae60", "#f2994a", "#9b51e0", "#56ccf2", "#219653", "#bb6bd9",
                "#f2c94c", "#4f4f4f", "#e67e22", "#16a085"];
let token = (typeof localStorage !== "undefined" && localStorage.getItem("det_token")) || "";
let seq = 0, epoch = "";
const ui = {expFilter: {text: "", state: "", project: "", archived: false}, selected: new Set(),
            runs: {sort: "id=desc", offset: 0, limit: 50}, followLogs: true};

// ------------------------------------------------------------------------------ helpers
async function api(path, opts = {}) {
  const h = {"Content-Type": "application/json"};
  if (token) h["Authorization"] = "Bearer " + token;
  const r = await fetch(path, Object.assign({headers: h}, opts));
  if (r.status === 401) { showLogin(); throw new Error("login required"); }
  const j = await r.json();
  if (!r.ok) throw new Error(j.error || r.status);
  return j;
}
const post = (path, body = {}) => api(path, {method: "POST", body: JSON.stringify(body)});
function esc(v) {
  return String(v === undefined || v === null ? "" : v).replace(/[&<>"']/g,
    c => ({"&": "&amp;", "<": "&lt;", ">": "&gt;", "\"": "&quot;", "'": "&#39;"})[c]);
}
function st(s) { return `<span class="st ${esc(s)}">${esc(s)}</span>`; }
function ts(t) { return t ? new Date(t * 1000).toLocaleString() : ""; }
function dur(a, b) {
  if (!a) return "";
  const s = Math.max(0, Math.round((b || Date.now() / 1000) - a));
  return s < 60 ? `${s}s` : s < 3600 ? `${Math.floor(s / 60)}m ${s % 60}s` : `${Math.floor(s / 3600)}h ${Math.floor(s % 3600 / 60)}m`;
}
function num(v) { return typeof v === "number" ? (Math.abs(v) >= 1e4 || (v !== 0 && Math.abs(v) < 1e-3) ? v.toExponential(3) : +v.toPrecision(5)) : esc(v); }
function bar(frac) { return `<div class="bar"><div style="width:${Math.round(100 * Math.min(1, frac || 0))}%"></div></div>`; }
function kv(obj) { return `<div class="kv">${Object.entries(obj).map(([k, v]) => `<div>${esc(k)}</div><div>${v}</div>`).join("")}</div>`; }
function tabs(base, items, cur) {
  return `<div class="tabs">${items.map(([id, label]) => `<a href="${base}/${id}" class="${id === cur ? "on" : ""}">${label}</a>`).join("")}</div>`;
}
function flatten(hp, prefix = "", out = {}) {  // nested hyperparameters -> {"a.b": v}
  for (const [k, v] of Object.entries(hp || {})) {
    if (v && typeof v === "object" && !Array.isArray(v)) flatten(v, prefix + k + ".", out);
    else out[prefix + k] = v;
  }
  return out;
}
function showErr(e) { if (String(e).indexOf("login") < 0) $("#err").textContent = String(e); }
async function act(path, body) { try { await post(path, body || {}); route(); } catch (e) { showErr(e); } }

function showLogin() {
  $("#view").innerHTML = `<div class="card" style="max-width:360px"><h2>Sign in</h2>
    <p><input id="u" placeholder="user" value="determined"></p><p><input id="p" type="password" placeholder="password"></p>
    <button class="primary" id="go">Sign in</button></div>`;
  $("#go").onclick = async () => {
    const r = await fetch("/api/v1/auth/login", {method: "POST", body: JSON.stringify({username: $("#u").value, password: $("#p").value})});
    const j = await r.json();
    if (!r.ok) { $("#err").textContent = j.error || "login failed"; return; }
    token = j.token; localStorage.setItem("det_token", token); whoami(); route();
  };
}

// ------------------------------------------------------------------------------ charts (inline SVG)
function axes(w, h, x0, x1, y0, y1, xlabel, ylabel) {
  return `<line x1="46" y1="${h - 22}" x2="${w - 8}" y2="${h - 22}" stroke="#aab"/>
    <line x1="46" y1="8" x2="46" y2="${h - 22}" stroke="#aab"/>
    <text x="2" y="14">${num(y1)}</text><text x="2" y="${h - 24}">${num(y0)}</text>
    <text x="46" y="${h - 8}">${num(x0)}</text><text x="${w - 70}" y="${h - 8}">${num(x1)}</text>
    ${xlabel ? `<text x="${w / 2 - 20}" y="${h - 8}">${esc(xlabel)}</text>` : ""}
    ${ylabel ? `<text x="50" y="16" style="font-weight:600">${esc(ylabel)}</text>` : ""}`;
}
function scale(lo, hi, a, b, log) {
  const f = log ? Math.log10 : (v => v);
  const L = f(lo), H = f(hi);
  return v => a + (b - a) * (H === L ? 0.5 : (f(v) - L) / (H - L));
}
function lineChart(series, opts = {}) {
  const w = opts.w || 640, h = opts.h || 230;
  const all = series.flatMap(s => s.pts).filter(p => isFinite(p[1]));
  if (!all.length) return `<i class="muted">no data yet</i>`;
  const xs = all.map(p => p[0]), ys = all.map(p => p[1]);
  const x0 = Math.min(...xs), x1 = Math.max(...xs), y0 = Math.min(...ys), y1 = Math.max(...ys);
  const logy = opts.logy && y0 > 0;
  const sx = scale(x0, x1, 50, w - 12), sy = scale(y0, y1, h - 24, 10, logy);
  let out = `<svg width="${w}" height="${h}">${axes(w, h, x0, x1, y0, y1, opts.xlabel || "batches", opts.ylabel)}`;
  series.forEach((s, i) => {
    const c = COLORS[i % COLORS.length];
    const pts = s.pts.filter(p => isFinite(p[1]));
    out += `<polyline fill="none" stroke="${c}" stroke-width="1.6" points="${pts.map(q => `${sx(q[0]).toFixed(1)},${sy(q[1]).toFixed(1)}`).join(" ")}"/>`;
    if (pts.length === 1) out += `<circle cx="${sx(pts[0][0])}" cy="${sy(pts[0][1])}" r="3" fill="${c}"/>`;
  });
  out += "</svg>";
  const legend = series.map((s, i) => `<span style="color:${COLORS[i % COLORS.length]}">&#9632; ${esc(s.name)}</span>`).join("");
  return out + `<div class="legend">${legend}</div>`;
}
function scatter(points, xlabel, ylabel, opts = {}) {  // points: [{x, y, label}]
  const w = opts.w || 420, h = opts.h || 260;
  const pts = points.filter(p => typeof p.x === "number" && typeof p.y === "number" && isFinite(p.x) && isFinite(p.y));
  if (!pts.length) return `<i class="muted">no numeric values for ${esc(xlabel)}</i>`;
  const x0 = Math.min(...pts.map(p => p.x)), x1 = Math.max(...pts.map(p => p.x));
  const y0 = Math.min(...pts.map(p => p.y)), y1 = Math.max(...pts.map(p => p.y));
  const logx = x0 > 0 && x1 / x0 > 100;
  const sx = scale(x0, x1, 50, w - 12, logx), sy = scale(y0, y1, h - 24, 10);
  let out = `<svg width="${w}" height="${h}">${axes(w, h, x0, x1, y0, y1, xlabel + (logx ? " (log)" : ""), ylabel)}`;
  for (const p of pts) out += `<circle cx="${sx(p.x).toFixed(1)}" cy="${sy(p.y).toFixed(1)}" r="4" fill="#2f80ed" fill-opacity=".7"><title>${esc(p.label)}: ${num(p.x)}, ${num(p.y)}</title></circle>`;
  return out + "</svg>";
}
function parallel(rows, dims, metric, opts = {}) {  // rows: [{vals: {dim: v}, metric}]
  const w = opts.w || Math.max(420, 130 * (dims.length + 1)), h = opts.h || 280;
  const axesAll = dims.concat([metric]);
  const get = (r, d) => d === metric ? r.metric : r.vals[d];
  const scales = {}, cats = {};
  for (const d of axesAll) {
    const vs = rows.map(r => get(r, d)).filter(v => v !== undefined && v !== null);
    if (vs.every(v => typeof v === "number")) {
      const lo = Math.min(...vs), hi = Math.max(...vs);
      scales[d] = scale(lo, hi, h - 24, 16, lo > 0 && hi / lo > 100);
      scales[d].lo = lo; scales[d].hi = hi;
    } else {
      cats[d] = [...new Set(vs.map(String))];
      const n = cats[d].length;
      scales[d] = v => 16 + (h - 40) * (n === 1 ? 0.5 : cats[d].indexOf(String(v)) / (n - 1));
    }
  }
  const ms = rows.map(r => r.metric).filter(v => typeof v === "number");
  const mlo = Math.min(...ms), mhi = Math.max(...ms);
  const color = v => { const t = mhi === mlo ? 0.5 : (v - mlo) / (mhi - mlo); return `hsl(${Math.round(220 - 200 * t)},75%,50%)`; };
  const xpos = i => 40 + (w - 80) * (axesAll.length === 1 ? 0.5 : i / (axesAll.length - 1));
  let out = `<svg width="${w}" height="${h}">`;
  for (const r of rows) {
    if (typeof r.metric !== "number") continue;
    const pts = axesAll.map((d, i) => { const v = get(r, d); return v === undefined || v === null ? null : `${xpos(i).toFixed(1)},${scales[d](v).toFixed(1)}`; }).filter(Boolean);
    out += `<polyline fill="none" stroke="${color(r.metric)}" stroke-opacity=".75" stroke-width="1.4" points="${pts.join(" ")}"><title>${esc(r.label)}</title></polyline>`;
  }
  axesAll.forEach((d, i) => {
    const x = xpos(i);
    out += `<line x1="${x}" y1="14" x2="${x}" y2="${h - 22}" stroke="#667"/><text x="${x - 30}" y="${h - 6}" style="font-weight:600">${esc(d)}</text>`;
    if (cats[d]) cats[d].forEach(c => { out += `<text x="${x + 3}" y="${scales[d](c) + 3}">${esc(c)}</text>`; });
    else { out += `<text x="${x + 3}" y="20">${num(scales[d].hi)}</text><text x="${x + 3}" y="${h - 26}">${num(scales[d].lo)}</text>`; }
  });
  return out + "</svg>";
}

// ------------------------------------------------------------------------------ experiments
async function viewExperiments() {
  const f = ui.expFilter;
  const d = await api("/api/v1/experiments" + (f.archived ? "" : "?archived=false"));
  const projects = [...new Set(d.experiments.map(e => `${e.workspace || ""}/${e.project || ""}`))].sort();
  const rows = d.experiments.filter(e =>
    (!f.text || (e.name || "").toLowerCase().includes(f.text.toLowerCase()) || (e.labels || []).some(l => l.includes(f.text)) || String(e.id) === f.text) &&
    (!f.state || e.state === f.state) && (!f.project || `${e.workspace || ""}/${e.project || ""}` === f.project)).reverse();
  const trs = rows.map(e => `<tr><td><input type="checkbox" data-exp="${e.id}" ${ui.selected.has(e.id) ? "checked" : ""}></td>
    <td><a href="#/experiments/${e.id}">${e.id}</a></td><td>${esc(e.name)}${e.unmanaged ? ' <span class="muted">(unmanaged)</span>' : ""}</td>
    <td>${st(e.state)}</td><td>${bar(e.progress)}</td><td>${esc(e.searcher_type)}</td><td>${e.num_trials}</td>
    <td>${esc(e.owner)}</td><td>${esc(e.workspace)} / ${esc(e.project)}</td><td>${esc((e.labels || []).join(", "))}</td>
    <td>${ts(e.start_time)}</td><td>${dur(e.start_time, e.end_time)}</td></tr>`).join("");
  const states = ["", "ACTIVE", "PAUSED", "COMPLETED", "CANCELED", "ERROR"];
  return `<div class="card"><h2>Experiments <span class="muted">${rows.length} of ${d.experiments.length}</span></h2>
    <div class="toolbar"><input id="f-text" placeholder="filter name / label / id" value="${esc(f.text)}">
      <select id="f-state">${states.map(s => `<option ${s === f.state ? "selected" : ""} value="${s}">${s || "any state"}</option>`).join("")}</select>
      <select id="f-project"><option value="">any project</option>${projects.map(p => `<option ${p === f.project ? "selected" : ""}>${esc(p)}</option>`).join("")}</select>
      <label class="muted"><input type="checkbox" id="f-arch" ${f.archived ? "checked" : ""}> archived</label>
      <span style="margin-left:16px" class="muted">selected:</span>
      ${["activate", "pause", "cancel", "kill", "archive", "unarchive"].map(a => `<button data-bulk="${a}">${a}</button>`).join("")}
    </div>
    <table><tr><th></th><th>ID</th><th>Name</th><th>State</th><th>Progress</th><th>Searcher</th><th>Trials</th><th>User</th>
    <th>Workspace / project</th><th>Labels</th><th>Started</th><th>Duration</th></tr>${trs}</table></div>`;
}
function bindExperiments() {
  const f = ui.expFilter;
  const on = (id, ev, fn) => { const el = $(id); if (el) el.addEventListener(ev, fn); };
  on("#f-text", "change", e => { f.text = e.target.value; route(); });
  on("#f-state", "change", e => { f.state = e.target.value; route(); });
  on("#f-project", "change", e => { f.project = e.target.value; route(); });
  on("#f-arch", "change", e => { f.archived = e.target.checked; route(); });
  document.querySelectorAll("[data-exp]").forEach(cb => cb.addEventListener("change", e => {
    const id = +e.target.dataset.exp; e.target.checked ? ui.selected.add(id) : ui.selected.delete(id); }));
  document.querySelectorAll("[data-bulk]").forEach(b => b.addEventListener("click", async e => {
    const a = e.target.dataset.bulk;
    for (const id of ui.selected) { try { await post(`/api/v1/experiments/${id}/${a}`); } catch (err) { showErr(err); } }
    ui.selected.clear(); route();
  }));
}

async function trialSeries(trials, group, metric) {
  const out = [];
  for (const t of trials.slice(0, 24)) {
    const m = await api(`/api/v1/trials/${t.id}/metrics?group=${group}`);
    const pts = m.metrics.filter(r => r.metrics && typeof r.metrics[metric] === "number").map(r => [r.steps_completed, r.metrics[metric]]);
    if (pts.length) out.push({name: `trial ${t.id}`, pts});
  }
  return out;
}

async function viewExperiment(id, tab) {
  tab = tab || "overview";
  const e = await api(`/api/v1/experiments/${id}`);
  const exp = e.experiment || e, cfg = e.config || {};
  const metric = (cfg.searcher || {}).metric, smaller = (cfg.searcher || {}).smaller_is_better !== false;
  const trials = (await api(`/api/v1/experiments/${id}/trials`)).trials;
  const head = `<div class="card"><h2>Experiment ${id}: ${esc(exp.name)} ${st(exp.state)}</h2>
    <div class="toolbar">${["activate", "pause", "cancel", "kill", "archive"].map(a => `<button onclick="act('/api/v1/experiments/${id}/${a}')">${a}</button>`).join("")}
    <span class="muted">${esc(exp.workspace)} / ${esc(exp.project)} &middot; ${esc(exp.owner)} &middot; started ${ts(exp.start_time)} &middot; ${dur(exp.start_time, exp.end_time)}</span></div>
    ${bar(exp.progress)}</div>`;
  const base = `#/experiments/${id}`;
  const t = tabs(base, [["overview", "Overview"], ["trials", "Trials"], ["hp", "Hyperparameters"], ["compare", "Compare"],
                        ["checkpoints", "Checkpoints"], ["config", "Configuration"], ["code", "Code"]], tab);
  let body = "";
  const best = trials.filter(x => typeof x.searcher_metric === "number")
    .sort((a, b) => smaller ? a.searcher_metric - b.searcher_metric : b.searcher_metric - a.searcher_metric)[0];
  if (tab === "overview") {
    body = `<div class="row"><div class="card"><h3>Validation ${esc(metric)}</h3>${lineChart(await trialSeries(trials, "validation", metric), {ylabel: metric})}</div>
      <div class="card" style="max-width:380px"><h3>Summary</h3>${kv({searcher: esc((cfg.searcher || {}).name), metric: esc(metric) + (smaller ? " (min)" : " (max)"),
        trials: trials.length, "active trials": trials.filter(x => x.state === "ACTIVE" || x.state === "RUNNING").length,
        "best trial": best ? `<a href="#/trials/${best.id}">${best.id}</a> (${num(best.searcher_metric)})` : "&ndash;",
        description: esc(exp.description), labels: esc((exp.labels || []).join(", ")), "parent": esc(exp.parent_id)})}</div></div>`;
  } else if (tab === "trials") {
    const hpKeys = [...new Set(trials.flatMap(x => Object.keys(flatten(x.hparams))))].sort();
    const rows = trials.map(x => { const hp = flatten(x.hparams); return `<tr><td><input type="checkbox" data-trial="${x.id}"></td>
      <td><a href="#/trials/${x.id}">${x.id}</a></td><td>${st(x.state)}</td>${hpKeys.map(k => `<td>${num(hp[k])}</td>`).join("")}
      <td>${num(x.searcher_metric)}</td><td>${x.total_batches}</td><td>${x.restarts}</td><td>${dur(x.start_time, x.end_time)}</td></tr>`; }).join("");
    body = `<div class="card"><div class="toolbar"><button class="primary" id="cmp">compare selected</button></div>
      <table><tr><th></th><th>Trial</th><th>State</th>${hpKeys.map(k => `<th>${esc(k)}</th>`).join("")}<th>${esc(metric)}</th><th>Batches</th><th>Restarts</th><th>Duration</th></tr>${rows}</table></div>`;
  } else if (tab === "hp") {
    const rows = trials.map(x => ({vals: flatten(x.hparams), metric: x.searcher_metric, label: `trial ${x.id}`}));
    const dims = [...new Set(rows.flatMap(r => Object.keys(r.vals)))].filter(k => new Set(rows.map(r => JSON.stringify(r.vals[k]))).size > 1);
    body = `<div class="card"><h3>Parallel coordinates (colour = ${esc(metric)})</h3>${dims.length ? parallel(rows, dims, metric) : '<i class="muted">no varying hyperparameters</i>'}</div>
      <div class="row">${dims.map(d => `<div class="card"><h3>${esc(d)} vs ${esc(metric)}</h3>${scatter(rows.map(r => ({x: r.vals[d], y: r.metric, label: r.label})), d, metric)}</div>`).join("")}</div>`;
  } else if (tab === "compare") {
    const names = (await api(`/api/v1/experiments/${id}/metric-names`)).metric_names || {};
    const q = new URLSearchParams(location.hash.split("?")[1] || "");
    const ids = (q.get("trials") || trials.slice(0, 8).map(x => x.id).join(",")).split(",").filter(Boolean).map(Number);
    const group = q.get("group") || "validation", m = q.get("metric") || metric;
    const opts = Object.entries(names).flatMap(([g, ms]) => ms.map(x => `<option value="${esc(g)}|${esc(x)}" ${g === group && x === m ? "selected" : ""}>${esc(g)} / ${esc(x)}</option>`)).join("");
    const chosen = trials.filter(x => ids.includes(x.id));
    const rows = chosen.map(x => `<tr><td><a href="#/trials/${x.id}">${x.id}</a></td><td>${st(x.state)}</td><td><code>${esc(JSON.stringify(x.hparams))}</code></td><td>${num(x.searcher_metric)}</td></tr>`).join("");
    body = `<div class="card"><div class="toolbar">metric <select id="cmp-metric">${opts}</select>
      <span class="muted">trials ${ids.join(", ")}</span></div>${lineChart(await trialSeries(chosen, group, m), {ylabel: m})}
      <table><tr><th>Trial</th><th>State</th><th>Hyperparameters</th><th>${esc(metric)}</th></tr>${rows}</table></div>`;
  } else if (tab === "checkpoints") {
    const ck = (await api(`/api/v1/experiments/${id}/checkpoints`)).checkpoints || [];
    body = `<div class="card"><table><tr><th>UUID</th><th>Trial</th><th>Batches</th><th>State</th><th>Reported</th><th>Metrics</th></tr>
      ${ck.slice().reverse().map(c => `<tr><td><code>${esc(c.uuid)}</code></td><td><a href="#/trials/${c.trial_id}">${c.trial_id}</a></td><td>${c.steps_completed}</td>
      <td>${st(c.state)}</td><td>${ts(c.report_time)}</td><td><code>${esc(JSON.stringify((c.metadata || {}).metrics || c.metrics || ""))}</code></td></tr>`).join("")}</table></div>`;
  } else if (tab === "config") {
    body = `<div class="card"><pre>${esc(JSON.stringify(cfg, null, 2))}</pre></div>`;
  } else if (tab === "code") {
    let tree = [];
    try { tree = (await api(`/api/v1/experiments/${id}/file_tree`)).files || []; } catch (err) { tree = []; }
    body = `<div class="card"><h3>Model definition</h3>${tree.length ? `<table><tr><th>Path</th><th>Size</th></tr>${tree.map(f => `<tr><td>${esc(f.path)}</td><td>${esc(f.content_length || f.size || "")}</td></tr>`).join("")}</table>` : '<i class="muted">no files</i>'}</div>`;
  }
  return head + t + body;
}
function bindExperiment(id, tab) {
  const cmp = $("#cmp");
  if (cmp) cmp.onclick = () => {
    const ids = [...document.querySelectorAll("[data-trial]:checked")].map(c => c.dataset.trial);
    location.hash = `#/experiments/${id}/compare?trials=${ids.join(",")}`;
  };
  const sel = $("#cmp-metric");
  if (sel) sel.onchange = e => {
    const [g, m] = e.target.value.split("|");
    const q = new URLSearchParams(location.hash.split("?")[1] || "");
    q.set("group", g); q.set("metric", m);
    location.hash = `#/experiments/${id}/compare?${q.toString()}`;
  };
}

// ------------------------------------------------------------------------------ trials
async function viewTrial(id) {
  const t = (await api(`/api/v1/trials/${id}`)).trial;
  const m = (await api(`/api/v1/trials/${id}/metrics`)).metrics;
  const groups = {};
  for (const r of m) for (const [k, v] of Object.entries(r.metrics || {})) if (typeof v === "number") {
    const g = r.group_name; (groups[g] = groups[g] || {}); (groups[g][k] = groups[g][k] || []).push([r.steps_completed, v]); }
  const charts = Object.entries(groups).map(([g, ms]) => `<div class="card"><h3>${esc(g)}</h3>${lineChart(Object.entries(ms).map(([name, pts]) => ({name, pts})))}</div>`).join("");
  const logs = (await api(`/api/v1/tasks/trial-${id}/logs?limit=500`)).logs.slice(-500).map(l => esc(l.log)).join("\n");
  const ck = (await api(`/api/v1/trials/${id}/checkpoints`)).checkpoints || [];
  const hp = flatten(t.hparams);
  return `<div class="card"><h2>Trial ${id} ${st(t.state)} <span class="muted">experiment <a href="#/experiments/${t.experiment_id}">${t.experiment_id}</a></span></h2>
    <div class="toolbar"><button onclick="act('/api/v1/trials/${id}/kill')">kill</button></div>
    <div class="row"><div class="card">${kv({batches: t.total_batches, restarts: t.restarts, seed: t.seed, started: ts(t.start_time),
      duration: dur(t.start_time, t.end_time), "searcher metric": num(t.searcher_metric), "latest checkpoint": `<code>${esc(t.latest_checkpoint)}</code>`})}</div>
    <div class="card"><h3>Hyperparameters</h3>${kv(Object.fromEntries(Object.entries(hp).map(([k, v]) => [k, num(v)])))}</div></div></div>
    <div class="row">${charts || '<div class="card"><i class="muted">no metrics yet</i></div>'}</div>
    <div class="card"><h3>Checkpoints</h3><table><tr><th>UUID</th><th>Batches</th><th>State</th><th>Reported</th></tr>
      ${ck.map(c => `<tr><td><code>${esc(c.uuid)}</code></td><td>${c.steps_completed}</td><td>${st(c.state)}</td><td>${ts(c.report_time)}</td></tr>`).join("")}</table></div>
    <div class="card"><h3>Logs <span class="muted">(last 500 lines, live)</span></h3><pre id="logs">${logs}</pre></div>`;
}

// ------------------------------------------------------------------------------ flat runs
async function viewRuns() {
  const r = ui.runs;
  const d = await post("/api/v1/runs", {sort: r.sort, offset: r.offset, limit: r.limit});
  const hpKeys = [...new Set(d.runs.flatMap(x => Object.keys(flatten(x.hparams))))].sort().slice(0, 8);
  const [sf, so] = r.sort.split("=");
  const th = (field, label) => `<th class="sort" data-sort="${field}">${label}${sf === field ? (so === "asc" ? " &#9650;" : " &#9660;") : ""}</th>`;
  const rows = d.runs.map(x => { const hp = flatten(x.hparams); return `<tr><td><a href="#/trials/${x.id}">${x.id}</a></td>
    <td><a href="#/experiments/${x.experiment_id}">${x.experiment_id}</a> ${esc(x.experiment_name)}</td><td>${st(x.state)}</td>
    <td>${esc(x.searcher_metric)}</td><td>${num(x.searcher_metric_value)}</td><td>${x.total_batches}</td>
    ${hpKeys.map(k => `<td>${num(hp[k])}</td>`).join("")}<td>${esc(x.workspace)} / ${esc(x.project)}</td><td>${ts(x.start_time)}</td></tr>`; }).join("");
  const p = d.pagination || {total: d.runs.length};
  return `<div class="card"><h2>Runs <span class="muted">${r.offset + 1}&ndash;${Math.min(r.offset + r.limit, p.total)} of ${p.total}</span></h2>
    <div class="toolbar"><button id="prev" ${r.offset === 0 ? "disabled" : ""}>&larr; prev</button><button id="next" ${r.offset + r.limit >= p.total ? "disabled" : ""}>next &rarr;</button></div>
    <table><tr>${th("id", "Run")}<th>Experiment</th>${th("state", "State")}<th>Metric</th>${th("searcher_metric_value", "Value")}${th("total_batches", "Batches")}
    ${hpKeys.map(k => `<th>${esc(k)}</th>`).join("")}<th>Workspace / project</th>${th("start_time", "Started")}</tr>${rows}</table></div>`;
}
function bindRuns() {
  const r = ui.runs;
  document.querySelectorAll("[data-sort]").forEach(h => h.addEventListener("click", e => {
    const f = e.currentTarget.dataset.sort, [sf, so] = r.sort.split("=");
    r.sort = `${f}=${sf === f && so === "desc" ? "asc" : "desc"}`; r.offset = 0; route(); }));
  const pv = $("#prev"), nx = $("#next");
  if (pv) pv.onclick = () => { r.offset = Math.max(0, r.offset - r.limit); route(); };
  if (nx) nx.onclick = () => { r.offset += r.limit; route(); };
}

// ------------------------------------------------------------------------------ projects
async function viewProjects(ws) {
  const wss = (await api("/api/v1/workspaces")).workspaces;
  if (ws === undefined) {
    return `<div class="card"><h2>Workspaces</h2><table><tr><th>ID</th><th>Name</th><th>Archived</th><th>Projects</th></tr>
      ${(await Promise.all(wss.map(async w => { const ps = (await api(`/api/v1/workspaces/${w.id}/projects`)).projects;
        return `<tr><td>${w.id}</td><td><a href="#/projects/${w.id}">${esc(w.name)}</a></td><td>${w.archived ? "yes" : ""}</td><td>${ps.map(p => esc(p.name)).join(", ")}</td></tr>`; }))).join("")}</table></div>`;
  }
  const w = wss.find(x => String(x.id) === String(ws)) || {};
  const ps = (await api(`/api/v1/workspaces/${ws}/projects`)).projects;
  const out = [];
  for (const p of ps) {
    const ex = (await api(`/api/v1/projects/${p.id}/experiments`)).experiments || [];
    out.push(`<div class="card"><h3>${esc(p.name)} <span class="muted">${esc(p.description)} ${p.archived ? "(archived)" : ""}</span></h3>
      <table><tr><th>ID</th><th>Name</th><th>State</th><th>Progress</th><th>Trials</th><th>User</th></tr>
      ${ex.map(e => `<tr><td><a href="#/experiments/${e.id}">${e.id}</a></td><td>${esc(e.name)}</td><td>${st(e.state)}</td><td>${bar(e.progress)}</td><td>${e.num_trials}</td><td>${esc(e.owner)}</td></tr>`).join("")}</table></div>`);
  }
  return `<div class="card"><h2>Workspace ${esc(w.name)}</h2><a href="#/projects">&larr; all workspaces</a></div>${out.join("")}`;
}

// ------------------------------------------------------------------------------ job queue
async function viewJobs() {
  const pools = (await api("/api/v1/resource-pools")).resource_pools;
  const parts = [];
  for (const p of pools) {
    const jobs = (await api(`/api/v1/job-queues?resource_pool=${encodeURIComponent(p.name)}`)).jobs;
    const sorted = jobs.slice().sort((a, b) => (a.allocated === b.allocated ? 0 : a.allocated ? -1 : 1) || (a.priority - b.priority) || (a.order - b.order));
    let pos = 0;
    parts.push(`<div class="card"><h3>${esc(p.name)} <span class="muted">${esc(p.scheduler_type)} &middot; ${p.slots_used} / ${p.slots_available} slots</span></h3>
      <table><tr><th>#</th><th>Allocation</th><th>Job</th><th>State</th><th>Slots</th><th>Priority</th><th>Weight</th><th>Preemptible</th></tr>
      ${sorted.map(j => `<tr><td>${j.allocated ? "" : ++pos}</td><td>${esc(j.alloc_id)}</td><td>${esc(j.job_id)}</td>
        <td>${st(j.preempting ? "STOPPING_CANCELED" : j.allocated ? "RUNNING" : "QUEUED")}</td><td>${j.slots}</td><td>${j.priority}</td><td>${num(j.weight)}</td><td>${j.preemptible ? "yes" : "no"}</td></tr>`).join("") || '<tr><td colspan="8" class="muted">empty</td></tr>'}</table></div>`);
  }
  return `<div class="card"><h2>Job queue</h2><span class="muted">running jobs first, then the queue in scheduling order (priority, submission)</span></div>` + parts.join("");
}

// ------------------------------------------------------------------------------ cluster
async function viewCluster() {
  const ag = (await api("/api/v1/agents")).agents, rp = (await api("/api/v1/resource-pools")).resource_pools;
  let agg = [];
  try {
    const end = new Date(), start = new Date(Date.now() - 7 * 86400e3);
    const d = (x) => x.toISOString().slice(0, 10);
    agg = (await api(`/api/v1/resources/allocation/aggregated?start_date=${d(start)}&end_date=${d(end)}&period=DAILY`)).resource_entries || [];
  } catch (e) { agg = []; }
  const pools = rp.map(p => `<div class="card" style="max-width:340px"><h3>${esc(p.name)}</h3>${kv({scheduler: esc(p.scheduler_type),
    "slots": `${p.slots_used} / ${p.slots_available} ${bar(p.slots_available ? p.slots_used / p.slots_available : 0)}`, agents: p.num_agents,
    workspaces: esc((p.bound_workspaces || []).join(", ") || "all")})}</div>`).join("");
  const agents = ag.map(a => `<tr><td>${esc(a.id)}</td><td>${esc(a.host)}</td><td>${esc(a.resource_pool)}</td><td>${a.gpu ? "GPU" : "CPU"}</td>
    <td><div class="slots">${(a.slot_owner || []).map((o, i) => `<div class="slot ${(a.disabled_slots || []).includes(i) ? "off" : o ? "busy" : ""}" title="${esc(o || "free")}">${i}</div>`).join("")}</div></td>
    <td>${a.used_slots} / ${a.slots}</td><td>${a.enabled ? "yes" : st("disabled")}</td>
    <td><button onclick="act('/api/v1/agents/${esc(a.id)}/${a.enabled ? "disable" : "enable"}')">${a.enabled ? "disable" : "enable"}</button></td></tr>`).join("");
  const usage = agg.map(r => `<tr><td>${esc(r.period_start || r.date || "")}</td><td>${num(r.seconds)}</td><td><code>${esc(JSON.stringify(r.by_username || r.by_user || {}))}</code></td></tr>`).join("");
  return `<div class="row">${pools}</div>
    <div class="card"><h2>Agents</h2><div class="legend"><span><span class="slot busy" style="display:inline-block"></span> busy</span>
      <span><span class="slot" style="display:inline-block"></span> free</span><span><span class="slot off" style="display:inline-block"></span> disabled</span></div>
      <table><tr><th>ID</th><th>Host</th><th>Pool</th><th>Type</th><th>Slots</th><th>Used</th><th>Enabled</th><th></th></tr>${agents}</table></div>
    <div class="card"><h2>Allocation (last 7 days)</h2>${usage ? `<table><tr><th>Day</th><th>Slot-seconds</th><th>By user</th></tr>${usage}</table>` : '<i class="muted">no usage recorded</i>'}</div>`;
}

// ------------------------------------------------------------------------------ tasks
async function viewTasks(id) {
  if (id) {
    const t = (await api(`/api/v1/tasks/${id}`)).task;
    const logs = (await api(`/api/v1/tasks/${id}/logs?limit=500`)).logs.map(l => esc(l.log)).join("\n");
    const px = t.proxy || {};
    const open = px.port && !px.tunnel ? `<a href="/proxy/${esc(id)}/" target="_blank">open</a>` : px.tunnel ? `<code>det shell open ${esc(id)}</code>` : "";
    return `<div class="card"><h2>${esc(t.type)} ${esc(id)} ${st(t.state)}</h2><div class="toolbar"><button onclick="act('/api/v1/tasks/${esc(id)}/kill')">kill</button> ${open}</div>
      ${kv({started: ts(t.start_time), ended: ts(t.end_time), "exit code": esc(t.exit_code), config: `<code>${esc(JSON.stringify(t.config))}</code>`})}</div>
      <div class="card"><h3>Logs</h3><pre id="logs">${logs}</pre></div>`;
  }
  const tasks = (await api("/api/v1/tasks")).tasks.slice().reverse();
  return `<div class="card"><h2>Tasks <span class="muted">notebooks, shells, TensorBoards, commands</span></h2>
    <table><tr><th>ID</th><th>Type</th><th>State</th><th>Started</th><th>Duration</th><th>Exit</th><th></th></tr>
    ${tasks.map(t => `<tr><td><a href="#/tasks/${esc(t.id)}">${esc(t.id)}</a></td><td>${esc(t.type)}</td><td>${st(t.state)}</td><td>${ts(t.start_time)}</td>
      <td>${dur(t.start_time, t.end_time)}</td><td>${esc(t.exit_code)}</td>
      <td>${t.state === "RUNNING" || t.state === "PENDING" ? `<button onclick="act('/api/v1/tasks/${esc(t.id)}/kill')">kill</button>` : ""}</td></tr>`).join("")}</table></div>`;
}

// ------------------------------------------------------------------------------ models
async function viewModels(name) {
  if (name) {
    const mdl = (await api(`/api/v1/models/${encodeURIComponent(name)}`)).model || {};
    const vs = (await api(`/api/v1/models/${encodeURIComponent(name)}/versions`)).model_versions || [];
    return `<div class="card"><h2>Model ${esc(name)}</h2>${kv({description: esc(mdl.description), labels: esc((mdl.labels || []).join(", ")),
      created: ts(mdl.creation_time), metadata: `<code>${esc(JSON.stringify(mdl.metadata || {}))}</code>`})}</div>
      <div class="card"><h3>Versions</h3><table><tr><th>Version</th><th>Checkpoint</th><th>Comment</th><th>Created</th></tr>
      ${vs.map(v => `<tr><td>${v.version}</td><td><code>${esc(v.checkpoint_uuid || (v.checkpoint || {}).uuid)}</code></td><td>${esc(v.comment)}</td><td>${ts(v.creation_time)}</td></tr>`).join("")}</table></div>`;
  }
  const ms = (await api("/api/v1/models")).models;
  return `<div class="card"><h2>Model registry</h2><table><tr><th>Name</th><th>Description</th><th>Labels</th><th>Created</th></tr>
    ${ms.map(m => `<tr><td><a href="#/models/${encodeURIComponent(m.name)}">${esc(m.name)}</a></td><td>${esc(m.description)}</td><td>${esc((m.labels || []).join(", "))}</td><td>${ts(m.creation_time)}</td></tr>`).join("")}</table></div>`;
}

// ------------------------------------------------------------------------------ admin
async function viewAdmin() {
  const safe = async (p, k) => { try { return (await api(p))[k] || []; } catch (e) { return null; } };
  const users = await safe("/api/v1/users", "users"), groups = await safe("/api/v1/groups", "groups");
  const roles = await safe("/api/v1/rbac/roles", "roles"), hooks = await safe("/api/v1/webhooks", "webhooks");
  const tpls = await safe("/api/v1/templates", "templates");
  let cfg = {};
  try { cfg = (await api("/api/v1/master/config")).config || {}; } catch (e) { cfg = {}; }
  const table = (rows, cols) => rows === null ? '<i class="muted">not permitted</i>' :
    `<table><tr>${cols.map(c => `<th>${esc(c)}</th>`).join("")}</tr>${rows.map(r => `<tr>${cols.map(c => `<td>${esc(typeof r[c] === "object" ? JSON.stringify(r[c]) : r[c])}</td>`).join("")}</tr>`).join("")}</table>`;
  return `<div class="row"><div class="card"><h2>Users</h2>${table(users, ["id", "username", "display_name", "admin", "active"])}</div>
    <div class="card"><h2>Groups</h2>${table(groups, ["id", "name", "members"])}</div></div>
    <div class="row"><div class="card"><h2>Roles</h2>${table(roles, ["name", "permissions"])}</div>
    <div class="card"><h2>Webhooks</h2>${table(hooks, ["id", "url", "webhook_type", "triggers"])}</div></div>
    <div class="card"><h2>Templates</h2>${table(tpls, ["name", "config"])}</div>
    <div class="card"><h2>Master configuration</h2><pre>${esc(JSON.stringify(cfg, null, 2))}</pre></div>`;
}

// ------------------------------------------------------------------------------ router
async function route() {
  const h = (location.hash || "#/experiments").split("?")[0];
  const parts = h.slice(2).split("/");
  const top = parts[0] || "experiments";
  document.querySelectorAll("header a").forEach(a => a.classList.toggle("on", a.dataset.nav === (top === "trials" ? "experiments" : top)));
  $("#err").textContent = "";
  try {
    let html, bind = null;
    if (top === "experiments" && parts[1]) { html = await viewExperiment(+parts[1], parts[2]); bind = () => bindExperiment(+parts[1], parts[2]); }
    else if (top === "trials") html = await viewTrial(+parts[1]);
    else if (top === "runs") { html = await viewRuns(); bind = bindRuns; }
    else if (top === "projects") html = await viewProjects(parts[1]);
    else if (top === "jobs") html = await viewJobs();
    else if (top === "cluster") html = await viewCluster();
    else if (top === "tasks") html = await viewTasks(parts[1] ? decodeURIComponent(parts[1]) : undefined);
    else if (top === "models") html = await viewModels(parts[1] ? decodeURIComponent(parts[1]) : undefined);
    else if (top === "admin") html = await viewAdmin();
    else { html = await viewExperiments(); bind = bindExperiments; }
    $("#view").innerHTML = html;
    const logs = $("#logs");
    if (logs) logs.scrollTop = logs.scrollHeight;
    if (bind) bind();
  } catch (e) { showErr(e); }
}
async function follow() {  // live updates: long-poll the master's event stream
  for (;;) {
    try {
      const d = await api(`/api/v1/stream?since=${seq}&timeout_seconds=25&epoch=${epoch}`);
      const changed = d.resync || d.events.length > 0;
      seq = d.last_seq; epoch = d.epoch || "";
      if (changed && !document.querySelector("input:focus,select:focus")) await route();
    } catch (e) { await new Promise(r => setTimeout(r, 3000)); }
  }
}
function whoami() { api("/api/v1/me").then(u => { $("#who").textContent = (u.user || {}).username || ""; }).catch(() => {}); }

if (typeof window !== "undefined" && !window.DAMD_TEST) {
  window.onhashchange = route;
  window.act = act;
  whoami();
  route().then(follow);
}
if (typeof module !== "undefined") module.exports = {flatten, lineChart, scatter, parallel, esc, num, dur, route};
