// Fleets: list, fleet detail (current instances with GPU health, every instance the fleet ever had
// with its termination reason, configuration) and instance detail across projects.
const healthText = (h) => {
  if (!h) return "";
  const t = h.thresholds || {};
  const parts = [h.status ? st(h.status) : (h.healthy === false ? st("failed") : "")];
  for (const k of ["hbm_tb_s", "bf16_tflops", "fp8_tflops", "rccl_busbw_gb_s"]) if (h[k] != null) parts.push(`${k} ${(+h[k]).toFixed(1)}` + (t[k] ? ` (min ${t[k]})` : ""));
  if (h.sku) parts.push(esc(h.sku));
  if (h.ran_at) parts.push("probed " + ago(h.ran_at));
  if (h.message) parts.push(`<span class="muted">${esc(h.message)}</span>`);
  return parts.filter(Boolean).join(" · ");
};
Object.assign(VIEWS, {
  async fleets(name, tab) {
    if (name) return VIEWS.fleet(name, tab);
    const fleets = await api(P("fleets/list"));
    const rows = fleets.map(f => {
      const live = f.instances.filter(i => !["terminated"].includes(i.status));
      const gpus = live.reduce((n, i) => n + (i.instance_type?.resources.gpus.length || 0), 0);
      const busy = live.reduce((n, i) => n + (i.busy_blocks || 0), 0), blocks = live.reduce((n, i) => n + (i.total_blocks || 1), 0);
      const conf = f.spec?.configuration || {};
      return [esc(f.name), conf.ssh_config ? "ssh" : "cloud", live.length, gpus, `${busy}/${blocks}`,
              [...new Set(live.map(i => i.backend))].map(esc).join(", "), st(f.status), ago(f.created_at)];
    });
    $("#main").innerHTML = `<h3>Fleets</h3><div class="row"><a href="#newfleet" class="muted">+ add SSH hosts</a> <a href="#apply" class="muted">+ new fleet (YAML)</a>
        <button id="fdel" disabled>Delete selected</button></div>` +
      table(["", "fleet", "kind", "instances", "GPUs", "busy blocks", "backends", "status", "created"],
            rows.map((r, i) => [`<input type="checkbox" class="fsel" value="${esc(fleets[i].name)}">`, ...r]), true);
    bindRows(fleets, f => location.hash = "#fleets/" + encodeURIComponent(f.name));
    const picked = () => $$(".fsel").filter(c => c.checked).map(c => c.value);
    $$(".fsel").forEach(c => { c.onclick = (e) => e.stopPropagation(); c.onchange = () => { $("#fdel").disabled = !picked().length; }; });
    $("#fdel").onclick = () => act(() => api(P("fleets/delete"), { names: picked() }),
      `Delete fleet(s) ${picked().join(", ")} and terminate their instances?`);
  },

  async fleet(name, tab = "instances") {
    const f = await api(P("fleets/get"), { name });
    const conf = f.spec?.configuration || {};
    $("#main").innerHTML = `<h3><a href="#fleets" class="muted">fleets</a> / ${esc(name)} ${st(f.status)}</h3>
      <div class="row muted">nodes ${esc(JSON.stringify(conf.nodes ?? ""))} · placement ${esc(conf.placement || "any")} ·
        ${conf.ssh_config ? "SSH fleet (" + (conf.ssh_config.hosts || []).length + " hosts)" : "cloud fleet"} · created ${ago(f.created_at)}
        <button id="delf">Delete fleet</button></div>
      ${tabs("ftabs", ["instances", "history", "configuration"], tab)}<div id="tab"></div>`;
    bindTabs("ftabs", t => location.hash = `#fleets/${encodeURIComponent(name)}/${t}`);
    $("#delf").onclick = () => act(() => api(P("fleets/delete"), { names: [name] }), `Delete fleet ${name} and terminate its instances?`);
    if (tab === "configuration") { $("#tab").innerHTML = `<pre>${esc(yamlish(conf).trimStart())}</pre>`; return; }
    if (tab === "history") {
      const all = await api("/api/instances/list", { project_names: [S.project], fleet_ids: [f.id], only_active: false, limit: 500 });
      $("#tab").innerHTML = `<p class="muted">Every instance this fleet has had, newest first.</p>` +
        table(["#", "instance", "backend", "region", "resources", "status", "reason", "price/h", "created"], all.map(i => [
          i.instance_num, `<a href="#instances/${encodeURIComponent(i.project_name)}/${encodeURIComponent(i.name)}">${esc(i.name)}</a>`, esc(i.backend), esc(i.region),
          i.instance_type ? res({ instance_type: i.instance_type }) : "", st(i.status), esc(i.termination_reason || ""),
          i.price != null ? "$" + i.price : "", ago(i.created)]));
      return;
    }
    $("#tab").innerHTML = table(["#", "instance", "backend", "region", "resources", "status", "blocks", "price/h", "GPU health", ""], f.instances.map(i => [
      i.instance_num, `<a href="#instances/${encodeURIComponent(S.project)}/${encodeURIComponent(i.name)}">${esc(i.name)}</a>`, esc(i.backend), esc(i.region),
      i.instance_type ? res({ instance_type: i.instance_type }) : "", st(i.status) + (i.unreachable ? ' <span class="err">unreachable</span>' : ""),
      `${i.busy_blocks}/${i.total_blocks ?? 1}`, i.price != null ? "$" + i.price : "", healthText(i.health),
      !["terminating", "terminated", "busy"].includes(i.status) ? `<a data-n="${i.instance_num}" class="deli muted">[delete]</a>` : ""]));
    $$("a.deli").forEach(a => a.onclick = () =>
      act(() => api(P("fleets/delete_instances"), { name, instance_nums: [+a.dataset.n] }), `Delete instance ${a.dataset.n}?`));
    timers.push(setInterval(() => { if (!location.hash.includes("/history") && !location.hash.includes("/configuration")) route(); }, 10000));
  },

  async instances(project, iname) {
    if (project && iname) return VIEWS.instance(project, iname);
    const f = JSON.parse(localStorage.getItem("dstack_inst_filter") || '{"active":true}');
    const inst = await api("/api/instances/list", { only_active: f.active, limit: 500 });
    const live = (i) => !["terminating", "terminated"].includes(i.status) && i.fleet_name;
    $("#main").innerHTML = `<h3>Instances (all projects)</h3><div class="row"><label><input type="checkbox" id="ia" ${f.active ? "checked" : ""}> active only</label></div>` +
      table(["instance", "project", "fleet", "backend", "region", "resources", "status", "blocks", "health", "price/h", "created", ""],
      inst.map(i => [`<a href="#instances/${encodeURIComponent(i.project_name)}/${encodeURIComponent(i.name)}">${esc(i.name)}</a>`, esc(i.project_name),
                     i.fleet_name ? `<a href="#fleets/${encodeURIComponent(i.fleet_name)}">${esc(i.fleet_name)}</a>` : "", esc(i.backend), esc(i.region),
                     i.instance_type ? res({ instance_type: i.instance_type }) : "", st(i.status), `${i.busy_blocks ?? 0}/${i.total_blocks ?? 1}`,
                     i.health ? (i.health.healthy === false ? `<span class="err">${esc(i.health.message || "unhealthy")}</span>` : "ok") +
                       (i.health.hbm_tb_s ? ` <span class="muted">${(+i.health.hbm_tb_s).toFixed(1)} TB/s</span>` : "") : "",
                     i.price != null ? "$" + i.price : "", ago(i.created),
                     live(i) ? `<a data-p="${esc(i.project_name)}" data-f="${esc(i.fleet_name)}" data-n="${i.instance_num}" class="deli muted">[terminate]</a>` : ""]));
    $("#ia").onchange = () => { f.active = $("#ia").checked; localStorage.setItem("dstack_inst_filter", JSON.stringify(f)); route(); };
    $$("a.deli").forEach(a => a.onclick = () => act(() => api(`/api/project/${encodeURIComponent(a.dataset.p)}/fleets/delete_instances`,
      { name: a.dataset.f, instance_nums: [+a.dataset.n] }), `Terminate instance ${a.dataset.n} of fleet ${a.dataset.f}?`));
  },

  async instance(project, iname) {
    const all = await api("/api/instances/list", { project_names: [project], only_active: false, limit: 1000 });
    const i = all.find(x => x.name === iname);
    if (!i) throw new Error(`instance ${iname} not found`);
    const r = i.instance_type?.resources;
    const runs = await api("/api/runs/list", { project_name: project, only_active: true, limit: 100 }).catch(() => []);
    const here = runs.filter(x => x.jobs.some(j => { const jpd = j.job_submissions.at(-1).job_provisioning_data;
      return jpd && i.hostname && jpd.hostname === i.hostname; }));
    $("#main").innerHTML = `<h3><a href="#instances" class="muted">instances</a> / ${esc(project)} / ${esc(iname)} ${st(i.status)}</h3>
      ${table(["field", "value"], [
        ["fleet", i.fleet_name ? `<a href="#fleets/${encodeURIComponent(i.fleet_name)}">${esc(i.fleet_name)}</a>` : ""], ["backend / region", `${esc(i.backend)} / ${esc(i.region)}`],
        ["hostname", esc(i.hostname || "")], ["resources", r ? res({ instance_type: i.instance_type }) + ` · ${(r.disk.size_mib / 1024) | 0} GB disk` : ""],
        ["GPUs", r ? r.gpus.map(g => `${esc(g.name)} ${(g.memory_mib / 1024) | 0}GB`).join(", ") : ""], ["blocks busy/total", `${i.busy_blocks ?? 0}/${i.total_blocks ?? 1}`],
        ["price/h", i.price != null ? "$" + i.price : ""], ["created", ago(i.created)], ["unreachable", i.unreachable ? '<span class="err">yes</span>' : "no"],
        ["termination", esc(i.termination_reason || "")], ["GPU health", healthText(i.health)]])}
      ${here.length ? `<h4>Active runs on this instance</h4>` + table(["run", "status"], here.map(x => [`<a href="#runs/${encodeURIComponent(x.run_spec.run_name)}">${esc(x.run_spec.run_name)}</a>`, st(x.status)])) : ""}
      ${i.health ? `<h4>Health probe</h4><pre>${esc(JSON.stringify(i.health, null, 2))}</pre>` : ""}`;
  },
});
