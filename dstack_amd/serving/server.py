"""OpenAI-compatible HTTP server of the serving engine (what a ``type: service`` replica runs).

Routes: ``GET /health``, ``GET /v1/models``, ``POST /v1/completions``, ``POST /v1/chat/completions``
(both with SSE streaming), ``GET /metrics`` (Prometheus text: running/waiting sequences, KV-cache
usage, token counters, TTFT) — the gateway / in-server model proxy
(``dstack_amd/proxy/lib/model_proxy.py``) forwards OpenAI requests here, and the service
autoscaler reads replica load next to amdsmi GPU utilisation.  Reference parity: the reference's
services run vLLM/TGI and its model proxy speaks the same OpenAI API
(reference ``src/dstack/_internal/proxy/lib/routers/model_proxy.py:27-102``).

The engine loop runs in its own thread; each HTTP request gets an asyncio queue that the engine
thread feeds through ``loop.call_soon_threadsafe``.
"""

from __future__ import annotations

import asyncio
import json
import time
import uuid

from fastapi import FastAPI, HTTPException, Request
from fastapi.responses import JSONResponse, PlainTextResponse, StreamingResponse

from dstack_amd.serving.engine import LLMEngine, SamplingParams
from dstack_amd.serving.tokenizer import load_tokenizer


class _Stream:
    """Incremental detokenization with stop strings for one engine request."""

    def __init__(self, tok, stop):
        self.tok = tok
        self.stop = [s for s in (stop or []) if s]
        self.ids: list[int] = []
        self.text = ""
        self.stopped = False

    def push(self, token) -> str:
        if token is None or self.stopped:
            return ""
        self.ids.append(token)
        full = self.tok.decode(self.ids)
        if full.endswith("�"):  # an incomplete UTF-8 sequence: wait for the next token
            return ""
        for s in self.stop:
            i = full.find(s)
            if i >= 0:
                full = full[:i]
                self.stopped = True
                break
        delta = full[len(self.text):]
        self.text = full
        return delta


def create_app(engine: LLMEngine, served_model_name: str, tokenizer=None) -> FastAPI:
    tok = tokenizer or load_tokenizer(engine.model.spec.path, engine.model.cfg.vocab_size)
    if not engine.eos_token_ids:
        engine.eos_token_ids = tuple(tok.eos_token_ids)
    state = dict(requests=0, ttft_sum=0.0, ttft_n=0, gen_tokens=0, prompt_tokens=0, started=time.time())

    from contextlib import asynccontextmanager

    @asynccontextmanager
    async def lifespan(app):
        engine.start()
        try:
            yield
        finally:
            engine.stop()

    app = FastAPI(title="dstack-amd serving", lifespan=lifespan)

    def _check_model(name):
        if name and name != served_model_name:
            raise HTTPException(404, detail={"message": f"model {name!r} does not exist", "type": "invalid_request_error",
                                             "code": "model_not_found"})

    def _params(body: dict, prompt_len: int, default_max: int) -> SamplingParams:
        max_ctx = engine.model.max_model_len
        if prompt_len >= max_ctx:
            raise HTTPException(400, detail={"message": f"prompt has {prompt_len} tokens; this model's maximum "
                                             f"context length is {max_ctx}", "type": "invalid_request_error"})
        mt = body.get("max_tokens") or body.get("max_completion_tokens") or default_max
        mt = max(1, min(int(mt), max_ctx - prompt_len))
        stop_ids = tuple(body.get("stop_token_ids") or ())
        t = body.get("temperature")
        return SamplingParams(max_tokens=mt, temperature=1.0 if t is None else float(t),
                              top_p=float(body.get("top_p") or 1.0), top_k=int(body.get("top_k") or 0),
                              seed=body.get("seed"), ignore_eos=bool(body.get("ignore_eos", False)),
                              stop_token_ids=stop_ids)

    def _submit(ids, params, stop):
        loop = asyncio.get_running_loop()
        q: asyncio.Queue = asyncio.Queue()

        def on_event(req, token, finished):
            loop.call_soon_threadsafe(q.put_nowait, (token, finished, req.finish_reason))

        try:
            req = engine.add_request(ids, params, on_event=on_event)
        except ValueError as e:
            raise HTTPException(400, detail={"message": str(e), "type": "invalid_request_error"}) from e
        state["requests"] += 1
        state["prompt_tokens"] += len(ids)
        return req, q, _Stream(tok, stop)

    async def _drain(req, q, st):
        """Yields (delta_text, finish_reason or None) until the request finishes.  A consumer that
        goes away early (client disconnect: GeneratorExit / CancelledError in the streaming body or
        the awaiting handler) aborts the request, so it stops decoding and frees its KV pages."""
        t0 = time.perf_counter()
        first = True
        done = False
        try:
            while True:
                token, finished, reason = await q.get()
                if first and token is not None:
                    state["ttft_sum"] += time.perf_counter() - t0
                    state["ttft_n"] += 1
                    first = False
                if token is not None:
                    state["gen_tokens"] += 1
                delta = st.push(token)
                if st.stopped and not finished:
                    engine.abort(req.id)
                    done = True
                    yield delta, "stop"
                    return
                if finished:
                    done = True
                    if reason == "abort":
                        reason = "stop"
                    if reason and reason.startswith("error"):
                        raise HTTPException(500, detail={"message": reason, "type": "server_error"})
                    yield delta, reason
                    return
                if delta:
                    yield delta, None
        finally:
            if not done:
                engine.abort(req.id)

    def _abort_all(subs):
        for _, (req, _q, _st) in subs:
            if not req.finished:
                engine.abort(req.id)

    def _prompts(body):
        p = body.get("prompt")
        if p is None:
            raise HTTPException(400, detail={"message": "prompt is required", "type": "invalid_request_error"})
        if isinstance(p, str):
            return [tok.encode(p)]
        if isinstance(p, list) and p and all(isinstance(x, int) for x in p):
            return [p]
        if isinstance(p, list) and all(isinstance(x, str) for x in p):
            return [tok.encode(x) for x in p]
        if isinstance(p, list) and all(isinstance(x, list) for x in p):
            return p
        raise HTTPException(400, detail={"message": "unsupported prompt format", "type": "invalid_request_error"})

    def _stop(body):
        s = body.get("stop")
        return [s] if isinstance(s, str) else list(s or [])

    @app.get("/health")
    async def health():
        return {"status": "ok"}

    @app.get("/v1/models")
    async def models():
        return {"object": "list", "data": [{"id": served_model_name, "object": "model", "created": int(state["started"]),
                                             "owned_by": "dstack-amd", "max_model_len": engine.model.max_model_len}]}

    @app.post("/v1/completions")
    async def completions(request: Request):
        body = await request.json()
        _check_model(body.get("model"))
        prompts = _prompts(body)
        n = int(body.get("n") or 1)
        rid = f"cmpl-{uuid.uuid4().hex[:24]}"
        created = int(time.time())
        # validate every prompt before submitting any: a 400 for prompt k must not leave prompts
        # 0..k-1 decoding with no consumer
        planned = []
        for p in prompts:
            for k in range(n):
                params = _params(body, len(p), 16)
                if params.seed is not None and n > 1:
                    params.seed = int(params.seed) + k
                planned.append((p, params))
        subs = []
        try:
            for p, params in planned:
                subs.append((p, _submit(p, params, _stop(body))))
        except BaseException:
            _abort_all(subs)
            raise
        want_lp = body.get("logprobs") is not None

        if body.get("stream"):
            async def gen():
                usage = {"prompt_tokens": 0, "completion_tokens": 0}
                try:
                    for idx, (p, (req, q, st)) in enumerate(subs):
                        async for delta, reason in _drain(req, q, st):
                            ch = {"index": idx, "text": delta, "logprobs": None, "finish_reason": reason}
                            yield "data: " + json.dumps({"id": rid, "object": "text_completion", "created": created,
                                                         "model": served_model_name, "choices": [ch]}) + "\n\n"
                        usage["prompt_tokens"] += len(p)
                        usage["completion_tokens"] += len(req.output_ids)
                finally:
                    _abort_all(subs)  # the client left mid-stream: later choices were never read
                if (body.get("stream_options") or {}).get("include_usage"):
                    usage["total_tokens"] = usage["prompt_tokens"] + usage["completion_tokens"]
                    yield "data: " + json.dumps({"id": rid, "object": "text_completion", "created": created,
                                                 "model": served_model_name, "choices": [], "usage": usage}) + "\n\n"
                yield "data: [DONE]\n\n"

            return StreamingResponse(gen(), media_type="text/event-stream")

        choices, pt, ct = [], 0, 0
        try:
            for idx, (p, (req, q, st)) in enumerate(subs):
                text, reason = "", None
                async for delta, r in _drain(req, q, st):
                    text += delta
                    reason = r or reason
                lp = None
                if want_lp:
                    lp = {"tokens": [tok.decode([t]) for t in req.output_ids], "token_logprobs": list(req.logprobs)}
                choices.append({"index": idx, "text": text, "logprobs": lp, "finish_reason": reason})
                pt += len(p)
                ct += len(req.output_ids)
        finally:
            _abort_all(subs)
        return {"id": rid, "object": "text_completion", "created": created, "model": served_model_name,
                "choices": choices, "usage": {"prompt_tokens": pt, "completion_tokens": ct, "total_tokens": pt + ct}}

    @app.post("/v1/chat/completions")
    async def chat(request: Request):
        body = await request.json()
        _check_model(body.get("model"))
        msgs = body.get("messages")
        if not isinstance(msgs, list) or not msgs:
            raise HTTPException(400, detail={"message": "messages must be a non-empty list", "type": "invalid_request_error"})
        ids = tok.encode(tok.apply_chat_template(msgs, add_generation_prompt=True), add_bos=True)
        params = _params(body, len(ids), engine.model.max_model_len - len(ids))
        req, q, st = _submit(ids, params, _stop(body))
        rid = f"chatcmpl-{uuid.uuid4().hex[:24]}"
        created = int(time.time())

        if body.get("stream"):
            async def gen():
                head = {"id": rid, "object": "chat.completion.chunk", "created": created, "model": served_model_name}
                yield "data: " + json.dumps(dict(head, choices=[{"index": 0, "delta": {"role": "assistant", "content": ""},
                                                                "finish_reason": None}])) + "\n\n"
                async for delta, reason in _drain(req, q, st):
                    d = {"content": delta} if delta else {}
                    yield "data: " + json.dumps(dict(head, choices=[{"index": 0, "delta": d,
                                                                    "finish_reason": reason}])) + "\n\n"
                if (body.get("stream_options") or {}).get("include_usage"):
                    u = {"prompt_tokens": len(ids), "completion_tokens": len(req.output_ids),
                         "total_tokens": len(ids) + len(req.output_ids)}
                    yield "data: " + json.dumps(dict(head, choices=[], usage=u)) + "\n\n"
                yield "data: [DONE]\n\n"

            return StreamingResponse(gen(), media_type="text/event-stream")

        text, reason = "", None
        async for delta, r in _drain(req, q, st):
            text += delta
            reason = r or reason
        return {"id": rid, "object": "chat.completion", "created": created, "model": served_model_name,
                "choices": [{"index": 0, "message": {"role": "assistant", "content": text}, "finish_reason": reason}],
                "usage": {"prompt_tokens": len(ids), "completion_tokens": len(req.output_ids),
                          "total_tokens": len(ids) + len(req.output_ids)}}

    @app.get("/metrics")
    async def metrics():
        m = engine.metrics()
        lines = []

        def g(name, help_, val, kind="gauge"):
            lines.extend([f"# HELP {name} {help_}", f"# TYPE {name} {kind}", f"{name} {val}"])

        g("dstack_serving_running", "sequences in the running batch", m["running"])
        g("dstack_serving_waiting", "sequences waiting for admission", m["waiting"])
        g("dstack_serving_kv_usage", "fraction of KV-cache pages in use", round(m["kv_usage"], 6))
        g("dstack_serving_kv_pages_total", "KV-cache pages (64 tokens each)", m["kv_pages_total"])
        g("dstack_serving_requests_total", "requests received", state["requests"], "counter")
        g("dstack_serving_prompt_tokens_total", "prompt tokens received", state["prompt_tokens"], "counter")
        g("dstack_serving_generation_tokens_total", "tokens generated", state["gen_tokens"], "counter")
        g("dstack_serving_preemptions_total", "sequences preempted (recomputed)", m["preemptions"], "counter")
        ttft = state["ttft_sum"] / state["ttft_n"] if state["ttft_n"] else 0.0
        g("dstack_serving_ttft_mean_seconds", "mean time to first token", round(ttft, 6))
        return PlainTextResponse("\n".join(lines) + "\n")

    @app.exception_handler(HTTPException)
    async def _http_error(request, exc: HTTPException):
        detail = exc.detail if isinstance(exc.detail, dict) else {"message": str(exc.detail)}
        return JSONResponse({"error": detail}, status_code=exc.status_code)

    return app
