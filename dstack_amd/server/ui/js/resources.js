// Apply (YAML -> plan -> apply), offers browser, volumes (+detail), gateways (+detail), models.
Object.assign(VIEWS, {
  async apply() {
    const fromRun = localStorage.getItem("dstack_apply_json");
    if (fromRun) { localStorage.removeItem("dstack_apply_json"); localStorage.setItem("dstack_apply_yaml", yamlish(JSON.parse(fromRun)).trimStart()); }
    const saved = localStorage.getItem("dstack_apply_yaml") || "type: task\nname: hello\ncommands:\n  - rocm-smi || echo no-gpu\nresources:\n  gpu: MI355X:1\n";
    $("#main").innerHTML = `<h3>Apply a configuration</h3>
      <p class="muted">Paste a run (task / service / dev-environment), fleet, volume or gateway configuration, plan it, then apply.</p>
      <textarea id="yaml" rows="14" style="width:100%;font-family:monospace">${esc(saved)}</textarea>
      <div class="row"><button id="plan">Plan</button><button class="primary" id="go" disabled>Apply</button>
        <label class="muted"><input type="checkbox" id="force"> force (replace a running run)</label><span id="aerr" class="err"></span></div>
      <div id="plan_out"></div>`;
    let pending = null;
    $("#plan").onclick = async () => {
      $("#aerr").textContent = ""; $("#plan_out").innerHTML = "…"; $("#go").disabled = true; pending = null;
      localStorage.setItem("dstack_apply_yaml", $("#yaml").value);
      try {
        const { type, configuration } = await api(P("configurations/parse"), { yaml: $("#yaml").value });
        if (["task", "service", "dev-environment"].includes(type)) {
          const run_spec = { run_name: configuration.name, repo_id: "ui", repo_data: { repo_type: "virtual" }, configuration, ssh_key_pub: "" };
          const plan = await api(P("runs/get_plan"), { run_spec, max_offers: 50 });
          const jp = plan.job_plans[0] || {};
          $("#plan_out").innerHTML = `<h4>Run plan</h4><div class="muted">${plan.job_plans.length} job(s) · ${jp.total_offers ?? 0} offers` +
            (jp.max_price != null ? ` · max price $${(+jp.max_price).toFixed(3)}/h` : "") +
            (plan.current_resource ? ` · <b>${esc(plan.action || "update")}</b> the existing run` : "") + `</div>` + offersTable(jp.offers || []) +
            `<details><summary class="muted">job specs</summary><pre>${esc(JSON.stringify(plan.job_plans.map(x => x.job_spec), null, 1))}</pre></details>`;
          pending = () => api(P("runs/apply"), { plan: { run_spec: plan.run_spec, current_resource: plan.current_resource }, force: $("#force").checked })
            .then(r => { location.hash = "#runs/" + encodeURIComponent(r.run_spec.run_name); });
        } else if (type === "fleet") {
          const spec = { configuration };
          const plan = await api(P("fleets/get_plan"), { spec });
          $("#plan_out").innerHTML = `<h4>Fleet plan</h4><div class="muted">${plan.total_offers} offers${plan.current_resource ? " · the fleet exists" : ""}</div>` + offersTable(plan.offers || []);
          pending = () => api(P("fleets/create"), { spec }).then(f => { location.hash = "#fleets/" + encodeURIComponent(f.name); });
        } else if (type === "volume") {
          const plan = await api(P("volumes/get_plan"), { spec: { configuration } }).catch(() => null);
          $("#plan_out").innerHTML = `<h4>Volume</h4><pre>${esc(yamlish(configuration).trimStart())}</pre>` + (plan?.offers ? offersTable(plan.offers) : "");
          pending = () => api(P("volumes/create"), { configuration }).then(v => { location.hash = "#volumes/" + encodeURIComponent(v.name); });
        } else if (type === "gateway") {
          $("#plan_out").innerHTML = `<h4>Gateway</h4><pre>${esc(yamlish(configuration).trimStart())}</pre>`;
          pending = () => api(P("gateways/create"), { configuration }).then(g => { location.hash = "#gateways/" + encodeURIComponent(g.name); });
        }
        $("#go").disabled = !pending;
      } catch (e) { $("#plan_out").innerHTML = ""; $("#aerr").textContent = e.message; }
    };
    $("#go").onclick = async () => { try { await pending(); } catch (e) { $("#aerr").textContent = e.message; } };
  },

  async offers() {
    const q = JSON.parse(localStorage.getItem("dstack_offers_q") || '{"gpu":"MI355X:8","spot":"auto","max":"","backend":""}');
    $("#main").innerHTML = `<h3>Offers</h3>
      <p class="muted">Every configured backend's offers for a GPU spec (live provider listings where the backend has one, the offline catalog otherwise).</p>
      <div class="row"><input id="gpu" value="${esc(q.gpu)}" placeholder="gpu, e.g. MI355X:8 or 192GB..:1..">
        <select id="spot">${["auto", "on-demand", "spot"].map(x => `<option ${x === q.spot ? "selected" : ""}>${x}</option>`).join("")}</select>
        <input id="max" value="${esc(q.max)}" placeholder="max $/h" size="8"><input id="bk" value="${esc(q.backend || "")}" placeholder="backends (comma)" size="14">
        <button class="primary" id="find">Find</button><span id="oerr" class="err"></span></div>
      <div id="olist"></div>`;
    $("#find").onclick = async () => {
      const qq = { gpu: $("#gpu").value.trim(), spot: $("#spot").value, max: $("#max").value.trim(), backend: $("#bk").value.trim() };
      localStorage.setItem("dstack_offers_q", JSON.stringify(qq));
      const configuration = { type: "task", commands: [":"], spot_policy: qq.spot, resources: qq.gpu ? { gpu: qq.gpu } : {} };
      if (qq.max) configuration.max_price = +qq.max;
      if (qq.backend) configuration.backends = qq.backend.split(",").map(x => x.trim()).filter(Boolean);
      $("#oerr").textContent = ""; $("#olist").innerHTML = "…";
      try {
        const plan = await api(P("runs/get_plan"), { run_spec: { repo_id: "ui", repo_data: { repo_type: "virtual" }, configuration, ssh_key_pub: "" }, max_offers: 200 });
        const jp = plan.job_plans[0];
        $("#olist").innerHTML = `<div class="muted">${jp.total_offers} offers${jp.max_price != null ? ` · up to $${(+jp.max_price).toFixed(3)}/h` : ""}</div>` + offersTable(jp.offers);
      } catch (e) { $("#olist").innerHTML = ""; $("#oerr").textContent = e.message; }
    };
    $("#find").onclick();
  },

  async volumes(name) {
    if (name) return VIEWS.volume(name);
    const v = await api(P("volumes/list"));
    $("#main").innerHTML = `<h3>Volumes</h3><div class="row"><a href="#apply" class="muted">+ new volume (YAML)</a></div>` +
      table(["name", "backend", "region", "size", "attached to", "status", "created", ""],
      v.map(x => [`<a href="#volumes/${encodeURIComponent(x.name)}">${esc(x.name)}</a>`, esc(x.configuration.backend), esc(x.configuration.region),
                  x.provisioning_data ? x.provisioning_data.size_gb + "GB" : (x.configuration.size ? esc(x.configuration.size) : ""),
                  x.attachment_data ? `attached${x.attachment_data.device_name ? " (" + esc(x.attachment_data.device_name) + ")" : ""}` : "",
                  st(x.status), ago(x.created_at), `<a data-v="${esc(x.name)}" class="delv muted">[delete]</a>`]));
    $$("a.delv").forEach(a => a.onclick = () => act(() => api(P("volumes/delete"), { names: [a.dataset.v] }), `Delete volume ${a.dataset.v}?`));
  },
  async volume(name) {
    const v = await api(P("volumes/get"), { name });
    $("#main").innerHTML = `<h3><a href="#volumes" class="muted">volumes</a> / ${esc(name)} ${st(v.status)}</h3>
      ${v.status_message ? `<p class="err">${esc(v.status_message)}</p>` : ""}
      ${table(["field", "value"], [["backend / region", `${esc(v.configuration.backend)} / ${esc(v.configuration.region)}`],
        ["volume id", esc(v.volume_id || v.provisioning_data?.volume_id || v.configuration.volume_id || "")], ["size", v.provisioning_data ? v.provisioning_data.size_gb + " GB" : esc(v.configuration.size || "")],
        ["external", v.external ? "yes" : "no"], ["created", ago(v.created_at)], ["owner", esc(v.user || "")]])}
      <h4>Attachment</h4>${v.attachment_data ? table(["device"], [[esc(v.attachment_data.device_name || "(no device name)")]]) : '<p class="muted">not attached</p>'}
      <h4>Configuration</h4><pre>${esc(yamlish(v.configuration).trimStart())}</pre>`;
  },

  async gateways(name) {
    if (name) return VIEWS.gateway(name);
    const g = await api(P("gateways/list"));
    $("#main").innerHTML = `<h3>Gateways</h3><div class="row"><a href="#apply" class="muted">+ new gateway (YAML)</a></div>` +
      table(["name", "backend", "region", "hostname", "domain", "default", "status", ""],
      g.map(x => [`<a href="#gateways/${encodeURIComponent(x.name)}">${esc(x.name)}</a>`, esc(x.backend), esc(x.region), esc(x.hostname), esc(x.wildcard_domain),
                  x.default ? "✓" : `<a data-g="${esc(x.name)}" class="defg muted">[make default]</a>`, st(x.status), `<a data-g="${esc(x.name)}" class="delg muted">[delete]</a>`]));
    $$("a.defg").forEach(a => a.onclick = () => act(() => api(P("gateways/set_default"), { name: a.dataset.g })));
    $$("a.delg").forEach(a => a.onclick = () => act(() => api(P("gateways/delete"), { names: [a.dataset.g] }), `Delete gateway ${a.dataset.g}?`));
  },
  async gateway(name) {
    const g = await api(P("gateways/get"), { name });
    const runs = await api("/api/runs/list", { project_name: S.project, only_active: true, limit: 100 }).catch(() => []);
    const services = runs.filter(r => r.service && String(r.service.url).includes(g.wildcard_domain || "\0"));
    $("#main").innerHTML = `<h3><a href="#gateways" class="muted">gateways</a> / ${esc(name)} ${st(g.status)}</h3>
      ${g.status_message ? `<p class="err">${esc(g.status_message)}</p>` : ""}
      ${table(["field", "value"], [["backend / region", `${esc(g.backend)} / ${esc(g.region)}`], ["hostname / ip", `${esc(g.hostname || "")} ${esc(g.ip_address || "")}`],
        ["wildcard domain", esc(g.wildcard_domain || "")], ["default", g.default ? "yes" : "no"], ["created", ago(g.created_at)]])}
      <div class="row"><input id="wd" placeholder="*.example.com wildcard domain" value="${esc(g.wildcard_domain || "")}"><button id="swd">Set domain</button></div>
      <h4>Services behind it</h4>${table(["run", "url", "status"], services.map(r => [`<a href="#runs/${encodeURIComponent(r.run_spec.run_name)}">${esc(r.run_spec.run_name)}</a>`,
        `<a href="${esc(r.service.url)}">${esc(r.service.url)}</a>`, st(r.status)]))}
      <h4>Configuration</h4><pre>${esc(yamlish(g.configuration || {}).trimStart())}</pre>`;
    $("#swd").onclick = () => act(() => api(P("gateways/set_wildcard_domain"), { name, wildcard_domain: $("#wd").value.trim() }));
  },

  async models(name) {
    if (name) return VIEWS.model(name);
    const r = await fetch(`/proxy/models/${encodeURIComponent(S.project)}/models`, { headers: { "Authorization": "Bearer " + S.token } }).then(r => r.json());
    const runs = await api("/api/runs/list", { project_name: S.project, only_active: true, limit: 100 });
    const byModel = Object.fromEntries(runs.filter(x => x.service && x.service.model).map(x => [x.service.model.name, x]));
    $("#main").innerHTML = `<h3>Models</h3>` + table(["model", "owner", "service run", "status", "replicas"], r.data.map(m => {
      const run = byModel[m.id];
      return [`<a href="#models/${encodeURIComponent(m.id)}">${esc(m.id)}</a>`, esc(m.owned_by),
              run ? `<a href="#runs/${encodeURIComponent(run.run_spec.run_name)}">${esc(run.run_spec.run_name)}</a>` : "",
              run ? st(run.status) : "", run ? String(new Set((run.jobs || []).filter(j => j.job_submissions.at(-1)?.status === "running").map(j => j.job_spec.replica_num)).size) : ""];
    })) + chatBox(r.data.map(m => m.id));
    bindChat();
  },

  async model(name) {
    // model details: the service run behind it, its replicas, the OpenAI-compatible endpoint, a chat
    const runs = await api("/api/runs/list", { project_name: S.project, only_active: false, limit: 100 });
    const run = runs.find(x => x.service && x.service.model && x.service.model.name === name);
    const m = run ? run.service.model : { name };
    const base = `${location.origin}/proxy/models/${encodeURIComponent(S.project)}`;
    const replicas = run ? (run.jobs || []).map(j => { const sub = j.job_submissions.at(-1) || {}; const jpd = sub.job_provisioning_data;
      return [String(j.job_spec.replica_num), st(sub.status), jpd ? esc(jpd.hostname || "") : "", res(jpd), ago(sub.submitted_at)]; }) : [];
    const conf = run ? run.run_spec.configuration : {};
    $("#main").innerHTML = `<h3><a href="#models" class="muted">models</a> / ${esc(name)}</h3>` +
      table(["field", "value"], [["format", esc(m.format || m.type || "openai")], ["endpoint", `<code>${esc(base)}</code>`],
        ["service run", run ? `<a href="#runs/${encodeURIComponent(run.run_spec.run_name)}">${esc(run.run_spec.run_name)}</a> ${st(run.status)}` : "<span class=muted>none</span>"],
        ["service url", run && run.service.url ? `<a href="${esc(run.service.url)}">${esc(run.service.url)}</a>` : ""],
        ["replicas (min..max)", conf.replicas ? esc(JSON.stringify(conf.replicas)) : "1"],
        ["scaling", conf.scaling ? `${esc(conf.scaling.metric)} target ${esc(conf.scaling.target)}` : "manual"],
        ["resources", conf.resources ? esc(yamlish(conf.resources).trim().replace(/\n/g, " ")) : ""]]) +
      `<h4>Replicas</h4>` + table(["replica", "status", "host", "resources", "submitted"], replicas) +
      `<h4>Use it</h4><pre>curl ${esc(base)}/chat/completions \\
  -H "Authorization: Bearer &lt;token&gt;" -H "Content-Type: application/json" \\
  -d '{"model": "${esc(name)}", "messages": [{"role": "user", "content": "Hello"}]}'</pre>` + chatBox([name]);
    bindChat();
  },
});

// OpenAI chat against the project's model proxy (shared by the models list and a model's page)
function chatBox(models) {
  return `<h4>Chat</h4><div class="row"><select id="m">${models.map(m => `<option>${esc(m)}</option>`).join("")}</select>
    <input id="q" size="60" placeholder="message"><input id="mt" size="5" value="256" title="max tokens"><button class="primary" id="send">Send</button></div><pre id="a"></pre>`;
}
function bindChat() {
  const history = [];
  $("#send").onclick = async () => {
    history.push({ role: "user", content: $("#q").value });
    $("#a").textContent = history.map(m => `${m.role}: ${m.content}`).join("\n\n") + "\n\nassistant: …";
    const d = await fetch(`/proxy/models/${encodeURIComponent(S.project)}/chat/completions`, { method: "POST",
      headers: { "Authorization": "Bearer " + S.token, "Content-Type": "application/json" },
      body: JSON.stringify({ model: $("#m").value, messages: history, max_tokens: +$("#mt").value || 256 }) }).then(r => r.json());
    const answer = d.choices ? d.choices[0].message.content : JSON.stringify(d, null, 1);
    history.push({ role: "assistant", content: answer });
    $("#a").textContent = history.map(m => `${m.role}: ${m.content}`).join("\n\n"); $("#q").value = "";
  };
}
