// Configuration forms without YAML: task, service, dev-environment, cloud fleet and volume.  Each form
// builds the same configuration mapping the YAML parser produces, shows it as YAML, and hands it to the
// apply page (plan -> apply), so every kind goes through the server's own validation and plan.
const FORM_KINDS = {
  task: [["name", "text", "train"], ["image", "text", "rocm/pytorch:rocm7.0_ubuntu22.04_py3.10_pytorch_release_2.7.1"],
         ["commands", "lines", "python train.py"], ["gpu", "text", "MI355X:8"], ["nodes", "int", "1"],
         ["env", "list", "HF_TOKEN, NCCL_DEBUG=INFO"], ["volumes", "list", "my-volume:/data"], ["max_duration", "text", "72h"],
         ["spot_policy", "choice:auto,on-demand,spot", ""], ["retry", "choice:,no-capacity,error,interruption", ""]],
  service: [["name", "text", "llama"], ["image", "text", "rocm/vllm:latest"], ["commands", "lines", "vllm serve meta-llama/Meta-Llama-3-70B --port 8000"],
            ["port", "int", "8000"], ["gpu", "text", "MI355X:8"], ["replicas", "text", "1..4"], ["scaling_metric", "choice:,rps,gpu_util", ""],
            ["scaling_target", "float", "10"], ["model", "text", "meta-llama/Meta-Llama-3-70B"], ["auth", "bool", ""], ["env", "list", "HF_TOKEN"]],
  "dev-environment": [["name", "text", "dev"], ["ide", "choice:vscode,cursor", ""], ["image", "text", ""], ["gpu", "text", "MI355X:1"],
                      ["init", "lines", "pip install -r requirements.txt"], ["inactivity_duration", "text", "2h"], ["volumes", "list", ""]],
  fleet: [["name", "text", "mi355x-cloud"], ["nodes", "text", "2 or 0..4"], ["gpu", "text", "MI355X:8"], ["placement", "choice:any,cluster", ""],
          ["backends", "list", "aws, azure"], ["regions", "list", ""], ["spot_policy", "choice:auto,on-demand,spot", ""],
          ["idle_duration", "text", "30m"], ["blocks", "text", "auto"]],
  volume: [["name", "text", "my-volume"], ["backend", "text", "aws"], ["region", "text", "us-east-1"], ["size", "text", "500GB"],
           ["volume_id", "text", "(an existing volume instead of a new one)"]],
};

function buildConfiguration(kind, vals) {
  const c = { type: kind };
  const put = (k, v) => { if (v !== "" && v != null && !(Array.isArray(v) && !v.length)) c[k] = v; };
  const res = (g) => g ? { gpu: g } : undefined;
  for (const [k, v] of Object.entries(vals)) {
    if (["gpu", "scaling_metric", "scaling_target"].includes(k)) continue;
    if (k === "nodes" && kind === "fleet") { const m = String(v).match(/^(\d+)\.\.(\d+)$/); put(k, m ? { min: +m[1], max: +m[2] } : v === "" ? "" : +v); continue; }
    if (k === "replicas" || k === "blocks") { put(k, /^\d+$/.test(v) ? +v : v); continue; }
    put(k, v);
  }
  put("resources", res(vals.gpu));
  if (kind === "service" && vals.scaling_metric) c.scaling = { metric: vals.scaling_metric, target: vals.scaling_target ?? 10 };
  return c;
}

Object.assign(VIEWS, {
  async new(kind = "task") {
    const fields = FORM_KINDS[kind];
    if (!fields) throw new Error(`unknown kind ${kind}`);
    const input = ([name, type, ph]) => {
      if (type.startsWith("choice:")) return `<select data-n="${name}" data-t="text">${type.slice(7).split(",").map(o => `<option>${esc(o)}</option>`).join("")}</select>`;
      if (type === "bool") return `<select data-n="${name}" data-t="bool"><option value="">-</option><option>true</option><option>false</option></select>`;
      if (type === "lines") return `<textarea data-n="${name}" data-t="lines" rows="4" cols="70" placeholder="${esc(ph)}"></textarea>`;
      return `<input data-n="${name}" data-t="${type}" size="50" placeholder="${esc(ph)}">`;
    };
    $("#main").innerHTML = `<h3>New ${esc(kind)}</h3><div class="row">${Object.keys(FORM_KINDS).map(k =>
        `<a href="#new/${k}" class="${k === kind ? "" : "muted"}">${k}</a>`).join(" · ")}</div>` +
      fields.map(f => `<div class="row"><label>${esc(f[0])}</label>${input(f)}</div>`).join("") +
      `<div class="row"><button id="fy">Show YAML</button><button class="primary" id="fa">Plan on the apply page</button><span id="ferr" class="err"></span></div>
      <pre id="fyaml" hidden></pre>`;
    const read = () => {
      const vals = {};
      $$("[data-n]").forEach(el => {
        const raw = el.value.trim(), t = el.dataset.t;
        if (!raw) return;
        vals[el.dataset.n] = t === "lines" ? raw.split("\n").map(x => x.trim()).filter(Boolean)
          : t === "list" ? raw.split(",").map(x => x.trim()).filter(Boolean)
          : t === "int" ? parseInt(raw) : t === "float" ? parseFloat(raw) : t === "bool" ? raw === "true" : raw;
      });
      return buildConfiguration(kind, vals);
    };
    $("#fy").onclick = () => { $("#fyaml").hidden = false; $("#fyaml").textContent = yamlish(read()).trimStart(); };
    $("#fa").onclick = () => {
      try { localStorage.setItem("dstack_apply_yaml", yamlish(read()).trimStart()); location.hash = "#apply"; }
      catch (e) { $("#ferr").textContent = e.message; }
    };
  },
});
