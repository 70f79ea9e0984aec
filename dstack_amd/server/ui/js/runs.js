// Runs: list (filters, keyset paging, auto-refresh) and run detail (overview by replica with every
// job submission, paged logs with older/newer/follow/download, metric charts, configuration).
const RUN_STATUSES = ["", "submitted", "provisioning", "pulling", "running", "terminating", "pending", "done", "failed", "terminated"];
Object.assign(VIEWS, {
  async runs(name, tab) {
    if (name) return VIEWS.run(name, tab);
    const f = JSON.parse(localStorage.getItem("dstack_runs_filter") || '{"active":false,"status":"","type":"","q":"","refresh":true}');
    // list preferences (the reference's table preferences): page size and visible columns
    const ALL_COLS = ["name", "type", "user", "backend", "resources", "price/h", "cost", "status", "submitted"];
    const pref = Object.assign({ page: 50, cols: ALL_COLS }, JSON.parse(localStorage.getItem("dstack_runs_prefs") || "{}"));
    const body = (extra = {}) => ({ project_name: S.project, limit: pref.page, only_active: f.active, ...extra });
    let runs = await api("/api/runs/list", body());
    const sel = new Set();  // selected run names (kept across refreshes)
    const shown = () => runs.filter(r => (!f.status || r.status === f.status) && (!f.type || r.run_spec.configuration.type === f.type) &&
      (!f.q || (r.run_spec.run_name + " " + r.user).toLowerCase().includes(f.q.toLowerCase())));
    const render = () => {
      const rows = shown();
      $("#main").innerHTML = `<h3>Runs <span class="muted">${rows.length} shown</span></h3><div class="row">
        <label><input type="checkbox" id="act" ${f.active ? "checked" : ""}> active only</label>
        <select id="fs">${RUN_STATUSES.map(s => `<option value="${s}" ${s === f.status ? "selected" : ""}>${s || "any status"}</option>`).join("")}</select>
        <select id="ft">${["", "task", "service", "dev-environment"].map(s => `<option value="${s}" ${s === f.type ? "selected" : ""}>${s || "any type"}</option>`).join("")}</select>
        <input id="fq" placeholder="name or user" value="${esc(f.q)}"><label><input type="checkbox" id="fr" ${f.refresh ? "checked" : ""}> auto-refresh</label>
        <a href="#apply" class="muted">+ new run</a> <a id="prefs" class="muted">[preferences]</a></div>
        <div class="row"><span class="muted" id="nsel">0 selected</span><button id="bstop" disabled>Stop</button>
          <button id="babort" disabled>Abort</button><button id="bdel" disabled>Delete</button></div>
        <div id="prefbox" class="row" hidden>page size <select id="pg">${[10, 25, 50, 100].map(n => `<option ${n === pref.page ? "selected" : ""}>${n}</option>`).join("")}</select>
          ${ALL_COLS.map(c => `<label><input type="checkbox" class="pc" value="${c}" ${pref.cols.includes(c) ? "checked" : ""}> ${c}</label>`).join(" ")}</div>` +
        table([`<input type="checkbox" id="selall">`, ...pref.cols], rows.map(r => {
          const j = r.latest_job_submission || {}; const jpd = j.job_provisioning_data;
          const cell = { name: esc(r.run_spec.run_name), type: esc(r.run_spec.configuration.type), user: esc(r.user), backend: jpd ? esc(jpd.backend) : "",
            resources: res(jpd), "price/h": jpd ? "$" + (+jpd.price).toFixed(2) : "", cost: "$" + (+r.cost || 0).toFixed(2),
            status: st(r.status) + (r.error ? ` <span class="err">${esc(r.error)}</span>` : ""), submitted: ago(r.submitted_at) };
          return [`<input type="checkbox" class="rsel" value="${esc(r.run_spec.run_name)}" ${sel.has(r.run_spec.run_name) ? "checked" : ""}>`,
                  ...pref.cols.map(c => cell[c])];
        }), true) + (runs.length && runs.length % pref.page === 0 ? `<div class="row"><button id="more">Load more</button></div>` : "");
      bindRows(rows, r => location.hash = "#runs/" + encodeURIComponent(r.run_spec.run_name));
      // bulk actions over the selected runs (the reference's run list: stop / abort / delete)
      const FINISHED = ["done", "failed", "terminated", "aborted"];
      const picked = () => runs.filter(r => sel.has(r.run_spec.run_name));
      const sync = () => {
        const p = picked();
        $("#nsel").textContent = `${p.length} selected`;
        $("#bstop").disabled = $("#babort").disabled = !p.some(r => !FINISHED.includes(r.status));
        $("#bdel").disabled = !p.length || !p.every(r => FINISHED.includes(r.status));
      };
      $$(".rsel").forEach(cb => { cb.onclick = (e) => e.stopPropagation();
        cb.onchange = () => { cb.checked ? sel.add(cb.value) : sel.delete(cb.value); sync(); }; });
      $("#selall").onclick = (e) => e.stopPropagation();
      $("#selall").onchange = () => { rows.forEach(r => $("#selall").checked ? sel.add(r.run_spec.run_name) : sel.delete(r.run_spec.run_name)); render(); };
      const bulk = (body, path, q) => act(() => api(P(path), { runs_names: picked().map(r => r.run_spec.run_name), ...body })
        .then(() => sel.clear()), q);
      $("#bstop").onclick = () => bulk({ abort: false }, "runs/stop");
      $("#babort").onclick = () => bulk({ abort: true }, "runs/stop", `Abort ${picked().length} run(s)?`);
      $("#bdel").onclick = () => bulk({}, "runs/delete", `Delete ${picked().length} run(s)?`);
      sync();
      const save = () => localStorage.setItem("dstack_runs_filter", JSON.stringify(f));
      const savePrefs = () => { localStorage.setItem("dstack_runs_prefs", JSON.stringify(pref)); route(); };
      $("#prefs").onclick = () => { $("#prefbox").hidden = !$("#prefbox").hidden; };
      $("#pg").onchange = () => { pref.page = +$("#pg").value; savePrefs(); };
      $$(".pc").forEach(cb => cb.onchange = () => { pref.cols = ALL_COLS.filter(c => $$(".pc").find(x => x.value === c).checked); savePrefs(); });
      $("#act").onchange = () => { f.active = $("#act").checked; save(); route(); };
      $("#fs").onchange = () => { f.status = $("#fs").value; save(); render(); };
      $("#ft").onchange = () => { f.type = $("#ft").value; save(); render(); };
      $("#fq").oninput = () => { f.q = $("#fq").value; save(); render(); $("#fq").focus(); $("#fq").setSelectionRange(f.q.length, f.q.length); };
      $("#fr").onchange = () => { f.refresh = $("#fr").checked; save(); route(); };
      if ($("#more")) $("#more").onclick = async () => {  // keyset page after the last run shown
        const last = runs.at(-1);
        runs = runs.concat(await api("/api/runs/list", body({ prev_submitted_at: last.submitted_at, prev_run_id: last.id })));
        render();
      };
    };
    render();
    if (f.refresh) timers.push(setInterval(async () => {
      if (document.activeElement === $("#fq")) return;
      const fresh = await api("/api/runs/list", body()).catch(() => null);
      if (fresh && runs.length <= pref.page && !document.activeElement?.classList.contains("rsel")) { runs = fresh; render(); }
    }, 5000));
  },

  async run(name, tab = "overview") {
    const r = await api(P("runs/get"), { run_name: name });
    const finished = ["done", "failed", "terminated", "aborted"].includes(r.status);
    const conf = r.run_spec.configuration;
    $("#main").innerHTML = `<h3><a href="#runs" class="muted">runs</a> / ${esc(name)} ${st(r.status)}</h3>
      <div class="row">${finished ? `<button id="del">Delete</button>` : `<button id="stop">Stop</button><button id="abort">Abort</button>`}
      ${r.service ? `<span class="muted">service: <a href="${esc(r.service.url)}">${esc(r.service.url)}</a>${r.service.model ? ` · model ${esc(r.service.model.name)} at ${esc(r.service.model.base_url)}` : ""}</span>` : ""}
      <span class="muted">${esc(conf.type)} · by ${esc(r.user)} · submitted ${ago(r.submitted_at)} · cost $${(+r.cost || 0).toFixed(2)}
      ${r.termination_reason ? " · reason: " + esc(r.termination_reason) : ""}</span>${r.error ? `<span class="err">${esc(r.error)}</span>` : ""}</div>
      ${tabs("rtabs", ["overview", "jobs", "logs", "metrics", "configuration"], tab)}<div id="tab"></div>`;
    bindTabs("rtabs", t => location.hash = `#runs/${encodeURIComponent(name)}/${t}`);
    if (finished) $("#del").onclick = () => act(() => api(P("runs/delete"), { runs_names: [name] }).then(() => location.hash = "#runs"), `Delete ${name}?`);
    else {
      $("#stop").onclick = () => act(() => api(P("runs/stop"), { runs_names: [name], abort: false }));
      $("#abort").onclick = () => act(() => api(P("runs/stop"), { runs_names: [name], abort: true }), `Abort ${name}?`);
    }
    return RUN_TABS[tab] ? RUN_TABS[tab](r, name) : RUN_TABS.overview(r, name);
  },
});

const jobLabel = (j) => `${j.job_spec.job_name} (replica ${j.job_spec.replica_num}, node ${j.job_spec.job_num})`;
const RUN_TABS = {
  overview(r, name) {
    const byReplica = {};
    r.jobs.forEach(j => (byReplica[j.job_spec.replica_num] ??= []).push(j));
    let html = "";
    for (const [rep, jobs] of Object.entries(byReplica)) {
      if (Object.keys(byReplica).length > 1) html += `<h4>Replica ${esc(rep)}</h4>`;
      html += table(["job", "submission", "status", "exit", "instance", "resources", "gpus", "started", "duration", "reason"],
        jobs.flatMap(j => j.job_submissions.slice().reverse().map((s, k) => {
          const jpd = s.job_provisioning_data, jrd = s.job_runtime_data || {};
          const end = s.finished_at ? ts(s.finished_at) : Date.now();
          return [k ? "" : esc(j.job_spec.job_name), "#" + s.submission_num + (k ? ' <span class="muted">retry</span>' : ""), st(s.status), s.exit_status ?? "",
                  jpd ? `${esc(jpd.backend)}/${esc(jpd.region)} ${esc(jpd.instance_id || "")}` : "", res(jpd), esc((jrd.gpu_indices || []).join(",")),
                  ago(s.submitted_at), dur((end - ts(s.submitted_at)) / 1000),
                  esc(s.termination_reason || "") + (s.termination_reason_message ? ` <span class="muted">${esc(s.termination_reason_message)}</span>` : "")];
        })));
    }
    const last = r.jobs.map(j => j.job_submissions.at(-1));
    const t = last[0]?.timings;
    if (t && t.submitted) html += `<h4>Start-up timeline <span class="muted">${esc(r.jobs[0].job_spec.job_name)}</span></h4>` +
      table(["stage", "s after submit"], Object.entries(t).filter(([k]) => k !== "submitted").sort((a, b) => a[1] - b[1]).map(([k, v]) => [esc(k), (v - t.submitted).toFixed(2)]));
    const ports = last.flatMap(s => Object.entries(s.job_runtime_data?.ports || {}).map(([c, h]) => `${c}→${h}`));
    if (ports.length) html += `<div class="muted">ports: ${esc(ports.join(", "))}</div>`;
    $("#tab").innerHTML = html;
    if (!["done", "failed", "terminated"].includes(r.status)) timers.push(setInterval(() => { if (location.hash.endsWith("/overview") || location.hash === "#runs/" + encodeURIComponent(name)) route(); }, 5000));
  },

  jobs(r) {
    // one section per job: what it runs (image, commands, env names, requirements) and where its
    // latest submission landed (instance, GPUs, ports, volumes), the full specs on demand
    $("#tab").innerHTML = r.jobs.map((j, i) => {
      const spec = j.job_spec, sub = j.job_submissions.at(-1) || {}, jpd = sub.job_provisioning_data, jrd = sub.job_runtime_data || {};
      const req = spec.requirements || {};
      return `<h4>${esc(jobLabel(j))} ${st(sub.status)}</h4>` + table(["field", "value"], [
        ["image", esc(spec.image_name || "")], ["commands", `<pre>${esc((spec.commands || []).join("\n"))}</pre>`],
        ["working dir", esc(spec.working_dir || "")], ["env", esc(Object.keys(spec.env || {}).join(", "))],
        ["requirements", esc(yamlish(req.resources || req).trim().replace(/\n/g, " "))],
        ["max duration", spec.max_duration ? dur(spec.max_duration) : "-"], ["retry", esc(JSON.stringify(spec.retry || null))],
        ["instance", jpd ? `${esc(jpd.backend)}/${esc(jpd.region)} ${esc(jpd.instance_id || "")} ${esc(jpd.hostname || "")}` : ""],
        ["resources", res(jpd)], ["GPU indices", esc((jrd.gpu_indices || []).join(","))],
        ["ports", esc(Object.entries(jrd.ports || {}).map(([c, h]) => `${c}→${h}`).join(", "))],
        ["volumes", esc((jrd.volume_names || spec.volumes || []).map(v => typeof v === "string" ? v : v.name || JSON.stringify(v)).join(", "))],
        ["submissions", String(j.job_submissions.length)]]) +
        `<details><summary class="muted">job spec (JSON)</summary><pre>${esc(JSON.stringify(spec, null, 1))}</pre></details>` +
        `<details><summary class="muted">latest submission (JSON)</summary><pre>${esc(JSON.stringify(sub, null, 1))}</pre></details>`;
    }).join("");
  },

  async logs(r, name) {
    const subs = r.jobs.flatMap(j => j.job_submissions.map(s => ({ j, s })));
    let pick = subs.length - 1;
    $("#tab").innerHTML = `<div class="row"><select id="ljob">${subs.map((x, i) => `<option value="${i}" ${i === pick ? "selected" : ""}>${esc(jobLabel(x.j))} #${x.s.submission_num}</option>`).join("")}</select>
      <label class="muted"><input type="checkbox" id="diag"> runner logs</label><label class="muted"><input type="checkbox" id="follow" checked> follow</label>
      <button id="older">Older</button><button id="dl">Download</button><span id="lstat" class="muted"></span></div><pre id="logs"></pre>`;
    let first = null, last = null, lines = [];
    const show = () => { const el = $("#logs"); const bottom = el.scrollTop + el.clientHeight >= el.scrollHeight - 8;
      el.textContent = lines.join(""); if (bottom || $("#follow").checked) el.scrollTop = el.scrollHeight; $("#lstat").textContent = `${lines.length} entries`; };
    const q = (extra) => api(P("logs/poll"), { run_name: name, job_submission_id: subs[pick].s.id, limit: 500, diagnose: $("#diag").checked, ...extra });
    const dec = (e) => { try { return decodeURIComponent(escape(atob(e.message))); } catch { return atob(e.message); } };
    const reset = async () => {  // newest page first, then follow forward
      lines = []; first = last = null;
      const d = await q({ descending: true });
      const page = d.logs.slice().reverse();
      lines = page.map(dec); if (page.length) { first = page[0].timestamp; last = page.at(-1).timestamp; }
      show();
    };
    const newer = async () => {
      if (!$("#follow").checked) return;
      const d = await q(last ? { start_time: last } : {});
      const fresh = d.logs.filter(e => !last || e.timestamp > last);
      if (fresh.length) { lines.push(...fresh.map(dec)); last = fresh.at(-1).timestamp; first ??= fresh[0].timestamp; show(); }
    };
    $("#older").onclick = async () => {
      if (!first) return;
      const d = await q({ descending: true, end_time: first });
      const page = d.logs.filter(e => e.timestamp < first).reverse();
      if (!page.length) { $("#lstat").textContent = "beginning of log"; return; }
      lines.unshift(...page.map(dec)); first = page[0].timestamp;
      const el = $("#logs"), h = el.scrollHeight; el.textContent = lines.join(""); el.scrollTop = el.scrollHeight - h;
    };
    $("#dl").onclick = async () => {  // the whole log, page by page
      let out = [], tok = null;
      for (let i = 0; i < 1000; i++) {
        const d = await q({ next_token: tok, limit: 1000 });
        out.push(...d.logs.map(dec));
        if (!d.logs.length || !d.next_token || d.next_token === tok) break;
        tok = d.next_token;
      }
      download(`${name}-${subs[pick].j.job_spec.job_name}-${subs[pick].s.submission_num}${$("#diag").checked ? "-runner" : ""}.log`, out.join(""));
    };
    $("#ljob").onchange = () => { pick = +$("#ljob").value; reset(); };
    $("#diag").onchange = reset;
    await reset();
    timers.push(setInterval(newer, 1500));
  },

  async metrics(r, name) {
    const jobs = r.jobs;
    $("#tab").innerHTML = `<div class="row"><select id="mjob">${jobs.map((j, i) => `<option value="${i}">${esc(jobLabel(j))}</option>`).join("")}</select>
      <select id="mwin">${[60, 180, 720].map(n => `<option value="${n}">${n} samples</option>`).join("")}</select></div><div id="charts" class="charts">…</div>`;
    const draw = async () => {
      const spec = jobs[+$("#mjob").value].job_spec;
      const m = await api(P(`metrics/job/${encodeURIComponent(name)}?replica_num=${spec.replica_num}&job_num=${spec.job_num}&limit=${$("#mwin").value}`), null, "GET");
      const series = m.metrics.filter(x => x.values.length);
      $("#charts").innerHTML = series.length ? series.map(x => chart(x.name, x.timestamps || x.values.map((_, i) => Date.now() - (x.values.length - i) * 10000),
                                                                   x.values, v => fmtMetric(x.name, v))).join("") : "no samples yet";
    };
    $("#mjob").onchange = draw; $("#mwin").onchange = draw;
    await draw();
    timers.push(setInterval(draw, 10000));
  },

  configuration(r) {
    const spec = r.run_spec;
    $("#tab").innerHTML = `<div class="row"><button id="copy">Copy as JSON</button><a href="#apply" class="muted" id="reapply">edit & re-apply</a></div>
      <pre>${esc(yamlish(spec.configuration).trimStart())}</pre>` +
      (spec.profile ? `<h4>Profile</h4><pre>${esc(yamlish(spec.profile).trimStart())}</pre>` : "") +
      `<h4>Repository</h4><pre>${esc(yamlish({ repo_id: spec.repo_id, repo_data: spec.repo_data, working_dir: spec.working_dir }).trimStart())}</pre>`;
    $("#copy").onclick = () => navigator.clipboard?.writeText(JSON.stringify(spec.configuration, null, 2));
    $("#reapply").onclick = () => localStorage.setItem("dstack_apply_json", JSON.stringify(spec.configuration));
  },
};
