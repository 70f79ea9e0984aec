// dstack-amd web UI core: REST client, router, shared widgets (tables, tabs, charts, forms).
// Views register themselves in VIEWS (one module per area: dashboard.js, runs.js, fleets.js, resources.js,
// admin.js, forms.js).
const PAGES = ["home", "runs", "new", "apply", "offers", "fleets", "instances", "volumes", "gateways", "models", "projects", "users", "secrets"];
const S = { token: localStorage.getItem("dstack_token"), project: localStorage.getItem("dstack_project") || "main", me: null };
const VIEWS = {};
const $ = (s) => document.querySelector(s);
const $$ = (s) => [...document.querySelectorAll(s)];
const esc = (x) => String(x ?? "").replace(/[&<>"]/g, c => ({"&":"&amp;","<":"&lt;",">":"&gt;",'"':"&quot;"}[c]));
const st = (x) => `<span class="st ${esc(x)}">${esc(x)}</span>`;
const ts = (t) => t ? Date.parse(t.endsWith("Z") || t.includes("+") ? t : t + "Z") : NaN;
const ago = (t) => { if (!t) return "-"; const s = (Date.now() - ts(t)) / 1000;
  return s < 60 ? `${s|0}s ago` : s < 3600 ? `${(s/60)|0}m ago` : s < 86400 ? `${(s/3600)|0}h ago` : new Date(ts(t)).toLocaleString(); };
const dur = (sec) => sec == null || isNaN(sec) ? "-" : sec < 90 ? `${sec.toFixed(1)}s` : sec < 5400 ? `${(sec/60).toFixed(1)}m` : `${(sec/3600).toFixed(1)}h`;
const timers = [];
function clearTimers() { while (timers.length) clearInterval(timers.pop()); }

async function api(path, body, method = "POST") {
  const r = await fetch(path, { method, headers: { "Authorization": "Bearer " + S.token, "Content-Type": "application/json" },
                                body: method === "GET" ? undefined : JSON.stringify(body ?? {}) });
  if (r.status === 401 || r.status === 403) { if (path.includes("get_my_user")) { logout(); } throw new Error("forbidden"); }
  const d = await r.json().catch(() => ({}));
  if (!r.ok) throw new Error((d.detail && (d.detail[0]?.msg || d.detail)) || r.statusText);
  return d;
}
const P = (p) => `/api/project/${encodeURIComponent(S.project)}/${p}`;

function logout() { localStorage.removeItem("dstack_token"); S.token = null; login(); }

function login() {
  $("#nav").innerHTML = ""; $("#who").textContent = "";
  $("#main").innerHTML = `<h3>Sign in</h3><div class="row"><input id="tok" size="48" placeholder="user token (printed by dstack server)">
    <button class="primary" id="go">Sign in</button></div><div id="lerr" class="err"></div>`;
  $("#go").onclick = async () => { S.token = $("#tok").value.trim(); localStorage.setItem("dstack_token", S.token);
    try { await boot(); } catch (e) { $("#lerr").textContent = e.message; } };
}

async function boot() {
  S.me = await api("/api/users/get_my_user");
  $("#who").innerHTML = `<a href="#account" class="muted">${esc(S.me.username)}${S.me.global_role === "admin" ? " (admin)" : ""}</a>`;
  const projects = await api("/api/projects/list");
  if (!projects.find(p => p.project_name === S.project) && projects.length) S.project = projects[0].project_name;
  $("#project").innerHTML = projects.map(p => `<option ${p.project_name === S.project ? "selected" : ""}>${esc(p.project_name)}</option>`).join("");
  $("#project").onchange = () => { S.project = $("#project").value; localStorage.setItem("dstack_project", S.project); route(); };
  window.onhashchange = route; route();
}

function route() {
  clearTimers();
  const [page, ...args] = (location.hash.slice(1) || "home").split("/");
  $("#nav").innerHTML = PAGES.map(p => `<a href="#${p}" class="${p === page ? "active" : ""}">${p}</a>`).join("") + `<a onclick="logout()">sign out</a>`;
  (VIEWS[page] || VIEWS.home)(...args.map(decodeURIComponent)).catch(e => $("#main").innerHTML = `<p class="err">${esc(e.message)}</p>`);
}

// ---- widgets ---------------------------------------------------------------------------------
function table(cols, rows, onclick) {
  return `<table><tr>${cols.map(c => `<th>${c}</th>`).join("")}</tr>${rows.map((r, i) =>
    `<tr class="${onclick ? "click" : ""}" data-i="${i}">${r.map(c => `<td>${c}</td>`).join("")}</tr>`).join("")}</table>`;
}
function bindRows(items, fn, scope = document) { scope.querySelectorAll("tr.click").forEach(tr => tr.onclick = () => fn(items[+tr.dataset.i])); }
function tabs(id, names, current) {  // -> html; clicking a tab sets location.hash "<base>/<tab>"
  return `<div class="tabs" id="${id}">${names.map(n => `<a class="tab ${n === current ? "active" : ""}" data-t="${n}">${n}</a>`).join("")}</div>`;
}
function bindTabs(id, onpick) { $$(`#${id} a.tab`).forEach(a => a.onclick = () => onpick(a.dataset.t)); }
function spark(values, w = 220, h = 36) {  // inline SVG line chart of one metric series
  if (!values || values.length < 2) return "";
  const lo = Math.min(...values), hi = Math.max(...values), span = hi - lo || 1;
  const pts = values.map((v, i) => `${(i / (values.length - 1) * w).toFixed(1)},${(h - (v - lo) / span * (h - 4) - 2).toFixed(1)}`);
  return `<svg width="${w}" height="${h}" style="vertical-align:middle"><polyline fill="none" stroke="#e4572e" stroke-width="1.5" points="${pts.join(" ")}"/></svg>`;
}
function chart(title, times, values, fmt, w = 460, h = 120) {  // labelled chart: min/max axis, first/last time
  if (!values || values.length < 2) return `<div class="chart"><div class="muted">${esc(title)}: no samples</div></div>`;
  const lo = Math.min(...values), hi = Math.max(...values), span = hi - lo || 1;
  const pts = values.map((v, i) => `${(40 + i / (values.length - 1) * (w - 50)).toFixed(1)},${(h - 18 - (v - lo) / span * (h - 30)).toFixed(1)}`);
  const T = (t) => new Date(typeof t === "string" ? ts(t) : t).toLocaleTimeString();
  const t0 = T(times[0]), t1 = T(times.at(-1));
  return `<div class="chart"><div>${esc(title)} <b>${esc(fmt(values.at(-1)))}</b></div><svg width="${w}" height="${h}">
    <line x1="40" y1="${h - 18}" x2="${w - 10}" y2="${h - 18}" stroke="#262b36"/><line x1="40" y1="12" x2="40" y2="${h - 18}" stroke="#262b36"/>
    <text x="2" y="16" fill="#8b93a1" font-size="10">${esc(fmt(hi))}</text><text x="2" y="${h - 20}" fill="#8b93a1" font-size="10">${esc(fmt(lo))}</text>
    <text x="40" y="${h - 4}" fill="#8b93a1" font-size="10">${esc(t0)}</text><text x="${w - 70}" y="${h - 4}" fill="#8b93a1" font-size="10">${esc(t1)}</text>
    <polyline fill="none" stroke="#e4572e" stroke-width="1.5" points="${pts.join(" ")}"/></svg></div>`;
}
const fmtMetric = (name, v) => name.includes("bytes_per_s") ? (v / 2 ** 30).toFixed(2) + " GB/s" : name.includes("bytes") ? (v / 2 ** 30).toFixed(1) + " GB" :
  name.includes("percent") ? v.toFixed(0) + " %" : name.includes("watts") ? v.toFixed(0) + " W" :
  name.includes("temperature") ? v.toFixed(0) + " °C" : (Math.abs(v) >= 1e6 ? v.toExponential(2) : String(+v.toFixed(3)));
const avail = (a) => `<span class="st ${a === "available" ? "running" : a === "unknown" ? "" : "failed"}">${esc(a)}</span>`;
function res(jpd) { if (!jpd) return ""; const r = jpd.instance_type.resources; const g = r.gpus || [];
  return `${r.cpus}xCPU ${(r.memory_mib/1024)|0}GB` + (g.length ? ` ${g.length}x${esc(g[0].name)}` : ""); }
function offersTable(offers) {
  return table(["backend", "region", "instance", "resources", "spot", "price/h", "availability"], offers.map(o =>
    [esc(o.backend), esc(o.region), esc(o.instance.name), res({ instance_type: o.instance }) + ` ${(o.instance.resources.disk.size_mib / 1024) | 0}GB disk`,
     o.instance.resources.spot ? "spot" : "", "$" + (+o.price).toFixed(3), avail(o.availability)]));
}
async function act(fn, confirmText) { if (confirmText && !confirm(confirmText)) return; try { await fn(); route(); } catch (e) { alert(e.message); } }
function download(name, text) {
  const a = document.createElement("a"); a.href = URL.createObjectURL(new Blob([text], { type: "text/plain" }));
  a.download = name; a.click(); setTimeout(() => URL.revokeObjectURL(a.href), 1000);
}
function yamlish(obj, ind = "") {  // readable YAML-like dump of a configuration (no library in the page)
  if (obj === null || obj === undefined) return "null";
  if (Array.isArray(obj)) return obj.length ? obj.map(v => `\n${ind}- ${typeof v === "object" && v !== null ? yamlish(v, ind + "  ").trimStart() : yamlish(v)}`).join("") : "[]";
  if (typeof obj === "object") { const e = Object.entries(obj).filter(([, v]) => v !== null && !(Array.isArray(v) && !v.length));
    return e.length ? e.map(([k, v]) => `\n${ind}${k}:${typeof v === "object" ? yamlish(v, ind + "  ") : " " + yamlish(v)}`).join("") : "{}"; }
  return typeof obj === "string" && (/[:#\n]/.test(obj) || !obj) ? JSON.stringify(obj) : String(obj);
}

// ---- form builder over the server's field descriptors (/api/backends/form_schema) --------------
const SECRET = /key|secret|token|password|pass_phrase|data|content/;
function formFields(fields, prefix = "") {
  return fields.map(f => {
    const id = prefix + f.name, label = `${esc(f.name)}${f.required ? " *" : ""}`;
    if (f.kind === "object") return `<fieldset><legend>${label}</legend>${formFields(f.fields, id + ".")}</fieldset>`;
    if (f.kind === "union") return `<fieldset><legend>${label}</legend><select data-union="${esc(id)}">${f.variants.map(v =>
        `<option>${esc(v.type)}</option>`).join("")}</select>${f.variants.map((v, i) =>
        `<div class="variant" data-for="${esc(id)}" data-v="${esc(v.type)}" ${i ? "hidden" : ""}>${formFields(v.fields, id + ".")}</div>`).join("")}</fieldset>`;
    if (f.kind === "bool") return `<div class="row"><label>${label}</label><select data-f="${esc(id)}" data-k="bool"><option value="">-</option><option>true</option><option>false</option></select></div>`;
    const ph = f.kind === "list" ? "comma separated" : f.kind === "map" ? "key=value, key=value" : f.help || "";
    const type = SECRET.test(f.name) && f.kind === "str" ? "password" : "text";
    const input = f.name === "data" || f.name === "key_content" ? `<textarea data-f="${esc(id)}" data-k="${f.kind}" rows="3" cols="60" placeholder="${esc(ph)}"></textarea>`
      : `<input data-f="${esc(id)}" data-k="${f.kind}" type="${type}" size="40" placeholder="${esc(ph)}">`;
    return `<div class="row"><label>${label}</label>${input}</div>`;
  }).join("");
}
function bindForm(root) {
  root.querySelectorAll("select[data-union]").forEach(sel => sel.onchange = () =>
    root.querySelectorAll(`.variant[data-for="${sel.dataset.union}"]`).forEach(d => d.hidden = d.dataset.v !== sel.value));
}
function readForm(root, type) {  // -> config mapping (only the fields filled in)
  const out = { type };
  const put = (path, v) => { const ks = path.split("."); let o = out; ks.slice(0, -1).forEach(k => o = o[k] ??= {}); o[ks.at(-1)] = v; };
  root.querySelectorAll("select[data-union]").forEach(sel => { if (!sel.closest(".variant[hidden]")) put(sel.dataset.union + ".type", sel.value); });
  root.querySelectorAll("[data-f]").forEach(el => {
    if (el.closest(".variant[hidden]")) return;
    const raw = el.value.trim(); if (!raw) return;
    const k = el.dataset.k;
    const v = k === "list" ? raw.split(",").map(x => x.trim()).filter(Boolean) : k === "map" ? Object.fromEntries(raw.split(",").map(x => x.split("=").map(y => y.trim())))
      : k === "bool" ? raw === "true" : k === "int" ? parseInt(raw) : k === "float" ? parseFloat(raw) : raw;
    put(el.dataset.f, v);
  });
  return out;
}
