// Overview (the landing page) and the SSH-fleet form: what an operator of an MI355X pool looks at
// first -- runs by status, GPUs in use per fleet, hosts whose GPU health probe or RCCL pre-flight
// failed, the newest runs -- and the on-prem path of adding 8xMI355X hosts without writing YAML.
// (reference: frontend/src/pages/Runs/List, Fleets/List, Instances/List -- this page summarises
// the same REST data in one view.)
const RUN_ACTIVE = ["submitted", "provisioning", "pending", "running", "terminating"];

function tally(items, key) {
  const out = {};
  for (const x of items) { const k = key(x); out[k] = (out[k] || 0) + 1; }
  return out;
}

Object.assign(VIEWS, {
  async home() {
    const [runs, fleets, gateways] = await Promise.all([
      api("/api/runs/list", { project_name: S.project, limit: 100, descending: true }).catch(() => []),
      api(P("fleets/list")).catch(() => []),
      api(P("gateways/list")).catch(() => []),
    ]);
    const active = runs.filter(r => RUN_ACTIVE.includes(r.status));
    const byStatus = tally(runs, r => r.status);
    const insts = fleets.flatMap(f => f.instances.filter(i => i.status !== "terminated").map(i => ({ ...i, fleet: f.name })));
    const gpus = insts.reduce((n, i) => n + (i.instance_type?.resources.gpus.length || 0), 0);
    // a block is one GPU slice of a host (blocks: auto on an 8-GPU node = 8 blocks)
    const busyGpus = insts.reduce((n, i) => { const g = i.instance_type?.resources.gpus.length || 0, tb = i.total_blocks || 1;
      return n + Math.round(g * (i.busy_blocks || 0) / tb); }, 0);
    const unhealthy = insts.filter(i => i.health && i.health.healthy === false);
    const card = (label, value, sub = "") => `<div class="chart" style="min-width:170px"><div class="muted">${esc(label)}</div>
      <div style="font-size:26px">${value}</div><div class="muted">${sub}</div></div>`;
    $("#main").innerHTML = `<h3>Overview <span class="muted">${esc(S.project)}</span></h3>
      <div class="charts">
        ${card("active runs", active.length, Object.entries(byStatus).map(([k, v]) => `${esc(k)} ${v}`).join(" · "))}
        ${card("fleets", fleets.length, `${insts.length} instances`)}
        ${card("GPUs in use", `${busyGpus} / ${gpus}`, gpus ? `${Math.round(100 * busyGpus / gpus)} %` : "")}
        ${card("unhealthy hosts", unhealthy.length ? `<span class="err">${unhealthy.length}</span>` : "0", "GPU probe / RCCL pre-flight")}
        ${card("gateways", gateways.length, gateways.filter(g => g.default).map(g => "default " + esc(g.name)).join(""))}
      </div>
      <div class="row"><a href="#apply">+ apply a configuration</a> <a href="#newfleet">+ add SSH hosts (fleet)</a> <a href="#offers">browse offers</a></div>
      <h4>GPU capacity by fleet</h4>` +
      table(["fleet", "instances", "GPUs", "busy blocks", "health"], fleets.map(f => {
        const live = insts.filter(i => i.fleet === f.name);
        const g = live.reduce((n, i) => n + (i.instance_type?.resources.gpus.length || 0), 0);
        const bad = live.filter(i => i.health && i.health.healthy === false).length;
        return [`<a href="#fleets/${encodeURIComponent(f.name)}">${esc(f.name)}</a>`, live.length, g,
                `${live.reduce((n, i) => n + (i.busy_blocks || 0), 0)}/${live.reduce((n, i) => n + (i.total_blocks || 1), 0)}`,
                bad ? `<span class="err">${bad} unhealthy</span>` : "ok"];
      })) +
      (unhealthy.length ? `<h4>Unhealthy hosts</h4>` + table(["instance", "fleet", "reason"], unhealthy.map(i => [
        `<a href="#instances/${encodeURIComponent(S.project)}/${encodeURIComponent(i.name)}">${esc(i.name)}</a>`, esc(i.fleet), healthText(i.health)])) : "") +
      `<h4>Newest runs</h4>` + table(["run", "type", "status", "GPUs", "submitted"], runs.slice(0, 10).map(r => {
        const conf = r.run_spec.configuration || {};
        const g = conf.resources?.gpu;
        return [`<a href="#runs/${encodeURIComponent(r.run_spec.run_name)}">${esc(r.run_spec.run_name)}</a>`, esc(conf.type),
                st(r.status), esc(typeof g === "object" && g ? JSON.stringify(g.count ?? g) : g ?? ""), ago(r.submitted_at)];
      }));
    timers.push(setInterval(() => { if ((location.hash.slice(1) || "home") === "home") route(); }, 15000));
  },

  // SSH fleet without YAML: hosts, user, private key -> fleets/get_plan (what would be created, which
  // hosts are already in another fleet) -> fleets/create.  blocks: auto splits each 8xMI355X host
  // into GPU blocks aligned to its xGMI topology.
  async newfleet() {
    $("#main").innerHTML = `<h3><a href="#fleets" class="muted">fleets</a> / add SSH hosts</h3>
      <div class="row"><label>name</label><input id="fn" placeholder="mi355x-pool"></div>
      <div class="row"><label>hosts</label><textarea id="fh" rows="4" cols="50" placeholder="one per line: 10.0.0.11 or user@10.0.0.11:2222"></textarea></div>
      <div class="row"><label>user</label><input id="fu" placeholder="ubuntu"><label>port</label><input id="fp" size="6" placeholder="22"></div>
      <div class="row"><label>private key</label><textarea id="fk" rows="4" cols="60" placeholder="-----BEGIN OPENSSH PRIVATE KEY-----"></textarea></div>
      <div class="row"><label>blocks per host</label><select id="fb"><option>auto</option><option>1</option><option>2</option><option>4</option><option>8</option></select>
        <label>placement</label><select id="fpl"><option>any</option><option>cluster</option></select>
        <label>private network</label><input id="fnet" placeholder="10.0.0.0/24 (optional)"></div>
      <div class="row"><button id="fplan">Plan</button><button class="primary" id="fgo" disabled>Create fleet</button><span id="ferr" class="err"></span></div>
      <div id="fout"></div>`;
    const spec = () => {
      const hosts = $("#fh").value.split("\n").map(x => x.trim()).filter(Boolean).map(h => {
        const m = h.match(/^(?:([^@]+)@)?([^:]+)(?::(\d+))?$/);
        if (!m) throw new Error(`cannot parse host ${h}`);
        const o = { hostname: m[2] };
        if (m[1]) o.user = m[1];
        if (m[3]) o.port = +m[3];
        return Object.keys(o).length === 1 ? o.hostname : o;
      });
      if (!hosts.length) throw new Error("at least one host");
      const ssh = { hosts };
      if ($("#fu").value.trim()) ssh.user = $("#fu").value.trim();
      if ($("#fp").value.trim()) ssh.port = +$("#fp").value.trim();
      if ($("#fk").value.trim()) ssh.ssh_key = { public: "", private: $("#fk").value.trim() + "\n" };
      if ($("#fnet").value.trim()) ssh.network = $("#fnet").value.trim();
      const b = $("#fb").value;
      return { configuration: { type: "fleet", name: $("#fn").value.trim() || null, ssh_config: ssh,
                                blocks: b === "auto" ? "auto" : +b, placement: $("#fpl").value } };
    };
    $("#fplan").onclick = async () => {
      $("#ferr").textContent = ""; $("#fgo").disabled = true;
      try {
        const plan = await api(P("fleets/get_plan"), { spec: spec() });
        $("#fout").innerHTML = `<h4>Plan</h4><pre>${esc(yamlish(plan).trimStart())}</pre>`;
        $("#fgo").disabled = false;
      } catch (e) { $("#ferr").textContent = e.message; }
    };
    $("#fgo").onclick = async () => {
      try {
        const f = await api(P("fleets/create"), { spec: spec() });
        location.hash = "#fleets/" + encodeURIComponent(f.name);
      } catch (e) { $("#ferr").textContent = e.message; }
    };
  },
});
