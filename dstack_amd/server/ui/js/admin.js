// Projects (members with user suggestions, backends: form built from the server's field descriptors
// with a credentials check and region picker, or YAML; the project's gateways; the CLI set-up
// command), users, secrets.
Object.assign(VIEWS, {
  async projects(name, tab) {
    if (name) return VIEWS.project(name, tab);
    const p = await api("/api/projects/list");
    $("#main").innerHTML = `<h3>Projects</h3>` + table(["project", "owner", "members", "backends"], p.map(x => [esc(x.project_name),
      esc(x.owner.username), x.members.map(m => `${esc(m.user.username)} (${esc(m.project_role)})`).join(", "), (x.backends || []).map(b => esc(b.name || b)).join(", ")]), true) +
      `<div class="row"><input id="np" placeholder="new project"><button id="cp">Create</button></div>`;
    bindRows(p, x => location.hash = "#projects/" + encodeURIComponent(x.project_name));
    $("#cp").onclick = () => api("/api/projects/create", { project_name: $("#np").value }).then(() => boot()).catch(e => alert(e.message));
  },

  async project(name, tab = "members") {
    const p = await api(`/api/projects/${encodeURIComponent(name)}/get`);
    $("#main").innerHTML = `<h3><a href="#projects" class="muted">projects</a> / ${esc(name)}</h3>
      <div class="muted">owner ${esc(p.owner.username)} · created ${ago(p.created_at)}</div>
      ${tabs("ptabs", ["members", "backends", "gateways", "cli", "settings"], tab)}<div id="tab"></div>`;
    bindTabs("ptabs", t => location.hash = `#projects/${encodeURIComponent(name)}/${t}`);
    return (PROJECT_TABS[tab] || PROJECT_TABS.members)(p, name);
  },

  async users(name) {
    if (name) return VIEWS.user(name);
    const u = await api("/api/users/list");
    $("#main").innerHTML = `<h3>Users</h3>` + table(["user", "role", "email", "active", "created", ""], u.map(x => [
      `<a href="#users/${encodeURIComponent(x.username)}">${esc(x.username)}</a>`, esc(x.global_role), esc(x.email), x.active ? "yes" : "no", ago(x.created_at),
      `<a data-u="${esc(x.username)}" class="tok muted">[new token]</a> <a data-u="${esc(x.username)}" data-r="${x.global_role === "admin" ? "user" : "admin"}" class="role muted">[make ${x.global_role === "admin" ? "user" : "admin"}]</a> <a data-u="${esc(x.username)}" class="delu muted">[delete]</a>`])) +
      `<div class="row"><input id="nu" placeholder="username"><input id="ne" placeholder="email (optional)"><select id="nr"><option>user</option><option>admin</option></select><button id="cu">Create</button><span id="tok" class="muted"></span></div>`;
    $("#cu").onclick = () => api("/api/users/create", { username: $("#nu").value, global_role: $("#nr").value, email: $("#ne").value || null })
      .then(d => { $("#tok").textContent = "token: " + d.creds.token; }).catch(e => alert(e.message));
    $$("a.tok").forEach(a => a.onclick = () => api("/api/users/refresh_token", { username: a.dataset.u })
      .then(d => alert(`new token for ${a.dataset.u}: ${d.creds.token}`)).catch(e => alert(e.message)));
    $$("a.role").forEach(a => a.onclick = () => act(() => api("/api/users/update", { username: a.dataset.u, global_role: a.dataset.r })));
    $$("a.delu").forEach(a => a.onclick = () => act(() => api("/api/users/delete", { users: [a.dataset.u] }), `Delete user ${a.dataset.u}?`));
  },
  async user(name) {
    const u = await api("/api/users/get_user", { username: name });
    const projects = await api("/api/projects/list");
    const mine = projects.filter(p => p.members.some(m => m.user.username === name));
    $("#main").innerHTML = `<h3><a href="#users" class="muted">users</a> / ${esc(name)}</h3>` +
      table(["field", "value"], [["global role", esc(u.global_role)], ["email", esc(u.email || "")], ["active", u.active ? "yes" : "no"], ["created", ago(u.created_at)]]) +
      `<div class="row"><input id="ue" placeholder="email" value="${esc(u.email || "")}"><label><input type="checkbox" id="ua" ${u.active ? "checked" : ""}> active</label>
        <button id="us">Save</button></div><h4>Projects</h4>` +
      table(["project", "role"], mine.map(p => [`<a href="#projects/${encodeURIComponent(p.project_name)}">${esc(p.project_name)}</a>`,
        esc(p.members.find(m => m.user.username === name).project_role)]));
    $("#us").onclick = () => act(() => api("/api/users/update", { username: name, global_role: u.global_role, email: $("#ue").value || null, active: $("#ua").checked }));
  },

  async account() {
    // the signed-in user's own page (the reference's user settings): role, token (shown on demand,
    // copy, refresh), projects and roles
    const me = await api("/api/users/get_my_user");
    const projects = await api("/api/projects/list");
    const mine = projects.filter(p => p.members.some(m => m.user.username === me.username));
    $("#main").innerHTML = `<h3>Account <span class="muted">${esc(me.username)}</span></h3>` +
      table(["field", "value"], [["global role", esc(me.global_role)], ["email", esc(me.email || "")], ["created", ago(me.created_at)],
        ["token", `<code id="mytok">••••••••</code> <a id="showtok" class="muted">[show]</a> <a id="copytok" class="muted">[copy]</a>`]]) +
      `<div class="row"><button id="reftok">Refresh token</button><span class="muted">the old token stops working; the CLI config needs the new one</span></div>
      <h4>Projects</h4>` + table(["project", "role", "owner"], mine.map(p => [`<a href="#projects/${encodeURIComponent(p.project_name)}">${esc(p.project_name)}</a>`,
        esc(p.members.find(m => m.user.username === me.username).project_role), esc(p.owner.username)])) +
      `<div class="row"><a onclick="logout()" class="muted">sign out</a></div>`;
    const token = () => me.creds?.token || S.token;
    $("#showtok").onclick = () => { $("#mytok").textContent = token(); };
    $("#copytok").onclick = () => navigator.clipboard?.writeText(token());
    $("#reftok").onclick = () => act(async () => {
      const d = await api("/api/users/refresh_token", { username: me.username });
      S.token = d.creds.token; localStorage.setItem("dstack_token", S.token);
      alert("new token: " + S.token);
    }, "Refresh your token?");
  },

  async secrets() {
    const s = await api(P("secrets/list"));
    $("#main").innerHTML = `<h3>Secrets <span class="muted">${esc(S.project)}</span></h3>` + table(["name", ""], s.map(x => [esc(x.name), `<a data-s="${esc(x.name)}" class="dels muted">[delete]</a>`])) +
      `<div class="row"><input id="sn" placeholder="NAME"><input id="sv" placeholder="value" type="password"><button id="sa">Add / update</button></div>
      <p class="muted">Secrets are interpolated into runs as <code>\${{ secrets.NAME }}</code> and encrypted at rest.</p>`;
    $("#sa").onclick = () => api(P("secrets/add"), { name: $("#sn").value, value: $("#sv").value }).then(() => route()).catch(e => alert(e.message));
    $$("a.dels").forEach(a => a.onclick = () => act(() => api(P("secrets/delete"), { secrets_names: [a.dataset.s] }), `Delete secret ${a.dataset.s}?`));
  },
});

const PROJECT_TABS = {
  members(p, name) {
    const roles = ["admin", "manager", "user"];
    const memberRow = (u = "", r = "user") => `<div class="row mrow"><input class="mu" list="known-users" value="${esc(u)}" placeholder="username">
      <select class="mr">${roles.map(x => `<option ${x === r ? "selected" : ""}>${x}</option>`).join("")}</select><a class="muted rm">[remove]</a></div>`;
    $("#tab").innerHTML = `<datalist id="known-users"></datalist><div id="members">${p.members.map(m => memberRow(m.user.username, m.project_role)).join("")}</div>
      <div class="row"><button id="addm">Add member</button><button class="primary" id="savem">Save members</button></div>`;
    // user suggestions (admins can list users; others type the name)
    api("/api/users/list").then(us => { $("#known-users").innerHTML = us.map(u => `<option value="${esc(u.username)}">`).join(""); }).catch(() => {});
    const bindRm = () => $$("a.rm").forEach(a => a.onclick = () => a.closest(".mrow").remove());
    bindRm();
    $("#addm").onclick = () => { $("#members").insertAdjacentHTML("beforeend", memberRow()); bindRm(); };
    $("#savem").onclick = () => act(() => api(`/api/projects/${encodeURIComponent(name)}/set_members`, { members:
      $$(".mrow").map(r => ({ username: r.querySelector(".mu").value.trim(), project_role: r.querySelector(".mr").value })).filter(m => m.username) }));
  },

  async backends(p, name) {
    const B = (x) => `/api/project/${encodeURIComponent(name)}/backends/${x}`;
    const schema = await api("/api/backends/form_schema");
    const types = Object.keys(schema).filter(t => t !== "dstack");
    $("#tab").innerHTML = table(["backend", "settings", ""], (p.backends || []).map(b => [esc(b.name), esc(JSON.stringify(b.config || {})).slice(0, 160),
        `<a data-b="${esc(b.name)}" class="yb muted">[yaml]</a> <a data-b="${esc(b.name)}" class="delb muted">[delete]</a>`])) +
      `<h4>Add a backend</h4><div class="row"><select id="bt">${types.map(t => `<option>${esc(t)}</option>`).join("")}</select>
        <label class="muted"><input type="checkbox" id="asyaml"> as YAML</label></div>
      <div id="bform"></div><div class="row"><button id="chk">Check credentials & list regions</button><button class="primary" id="addb">Add backend</button>
        <span id="berr" class="err"></span></div><div id="bregions"></div>`;
    const renderForm = () => {
      if ($("#asyaml").checked) {
        $("#bform").innerHTML = `<textarea id="by" rows="8" cols="70" placeholder="type: vultr&#10;regions: [ewr]&#10;creds:&#10;  type: api_key&#10;  api_key: ..."></textarea>`;
      } else { $("#bform").innerHTML = formFields(schema[$("#bt").value]); bindForm($("#bform")); }
      $("#bregions").innerHTML = ""; $("#berr").textContent = "";
    };
    const current = () => {
      const conf = readForm($("#bform"), $("#bt").value);
      const picked = $$("#bregions input:checked").map(x => x.value);
      if (picked.length) conf[$("#bt").value === "azure" ? "locations" : "regions"] = picked;
      return conf;
    };
    $("#bt").onchange = renderForm; $("#asyaml").onchange = renderForm; renderForm();
    $("#chk").onclick = async () => {
      $("#berr").textContent = ""; $("#bregions").innerHTML = "…";
      try {
        const v = await api("/api/backends/config_values", current());
        $("#bregions").innerHTML = `<p class="muted">credentials ok${v.default_creds ? " · default credentials available" : ""} — regions:</p>` +
          v.regions.values.map(r => `<label class="chip"><input type="checkbox" value="${esc(r.value)}" ${v.regions.selected.includes(r.value) ? "checked" : ""}> ${esc(r.label)}</label>`).join(" ");
      } catch (e) { $("#bregions").innerHTML = ""; $("#berr").textContent = e.message; }
    };
    $("#addb").onclick = () => act(() => $("#asyaml").checked ? api(B("create_yaml"), { config_yaml: $("#by").value }) : api(B("create"), current()))
      .then(() => { location.hash = `#projects/${encodeURIComponent(name)}/backends`; });
    $$("a.delb").forEach(a => a.onclick = () => act(() => api(B("delete"), { backends_names: [a.dataset.b] }), `Delete backend ${a.dataset.b}?`));
    $$("a.yb").forEach(a => a.onclick = async () => {
      const y = await api(B(`${encodeURIComponent(a.dataset.b)}/get_yaml`));
      $("#asyaml").checked = true; renderForm(); $("#by").value = y.config_yaml;
      $("#addb").textContent = "Update backend";
      $("#addb").onclick = () => act(() => api(B("update_yaml"), { config_yaml: $("#by").value }));
    });
  },

  async gateways(p, name) {
    // the project's gateways (service endpoints with TLS and autoscaling), default first; a new one
    // from a short form (the full configuration is on the apply page)
    const G = (x) => `/api/project/${encodeURIComponent(name)}/gateways/${x}`;
    const gws = await api(G("list"));
    const backends = (p.backends || []).map(b => b.name || b);
    $("#tab").innerHTML = table(["gateway", "backend / region", "hostname", "wildcard domain", "default", "status", ""], gws.map(g => [
        `<a href="#gateways/${encodeURIComponent(g.name)}">${esc(g.name)}</a>`, `${esc(g.backend)} / ${esc(g.region)}`, esc(g.hostname || ""),
        esc(g.wildcard_domain || ""), g.default ? "yes" : `<a data-g="${esc(g.name)}" class="defg muted">[make default]</a>`, st(g.status),
        `<a data-g="${esc(g.name)}" class="delg muted">[delete]</a>`])) +
      `<h4>Add a gateway</h4><div class="row"><input id="gn" placeholder="name"><select id="gb">${backends.map(b => `<option>${esc(b)}</option>`).join("")}</select>
        <input id="gr" placeholder="region"><input id="gd" placeholder="*.example.com domain (optional)"><label><input type="checkbox" id="gdef"> default</label>
        <button class="primary" id="gadd">Create</button><span id="gerr" class="err"></span></div>`;
    $$("a.defg").forEach(a => a.onclick = () => act(() => api(G("set_default"), { name: a.dataset.g })));
    $$("a.delg").forEach(a => a.onclick = () => act(() => api(G("delete"), { names: [a.dataset.g] }), `Delete gateway ${a.dataset.g}?`));
    $("#gadd").onclick = async () => {
      const configuration = { type: "gateway", name: $("#gn").value.trim() || null, backend: $("#gb").value, region: $("#gr").value.trim(),
                              default: $("#gdef").checked };
      if ($("#gd").value.trim()) configuration.domain = $("#gd").value.trim();
      try { await api(G("create"), { configuration }); route(); } catch (e) { $("#gerr").textContent = e.message; }
    };
  },

  async cli(p, name) {
    // the CLI / Python API set-up for this project: the same server URL and the signed-in user's token
    const url = location.origin;
    const cmd = `dstack config --url ${url} --project ${name} --token ${S.token}`;
    $("#tab").innerHTML = `<p class="muted">Run this to point the CLI at this project (it writes ~/.dstack/config.yml):</p>
      <pre id="clicmd">${esc(cmd)}</pre><div class="row"><button id="copy">Copy</button><span id="copied" class="muted"></span></div>
      <p class="muted">Python API:</p><pre>${esc(`from dstack_amd.api import Client\nclient = Client.from_config(project_name="${name}")\nprint([r.name for r in client.runs.list()])`)}</pre>`;
    $("#copy").onclick = () => navigator.clipboard.writeText(cmd).then(() => { $("#copied").textContent = "copied"; }).catch(e => alert(e.message));
  },

  settings(p, name) {
    $("#tab").innerHTML = `<h4>Default gateway</h4><p class="muted">Set on the <a href="#gateways">gateways</a> page.</p>
      <h4>SSH key</h4><pre>${esc(p.ssh_public_key || "(hidden)")}</pre>
      <h4>Danger zone</h4><button id="delp">Delete project</button>`;
    $("#delp").onclick = () => act(() => api("/api/projects/delete", { projects_names: [name] }).then(() => { location.hash = "#projects"; return boot(); }),
      `Delete project ${name} and its runs, fleets and volumes?`);
  },
};
