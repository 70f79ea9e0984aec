"""OpenAI-compatible model proxy shared by the in-server proxy and the gateway (reference:
``P/lib/routers/model_proxy.py:27-102``, ``clients/openai.py:16-67``, ``clients/tgi.py:24-208``).

``format: openai`` services are passed through (``/v1/chat/completions``); ``format: tgi`` services
are adapted: chat messages are rendered with the model's chat template (Jinja) into a prompt for
TGI's ``/generate`` / ``/generate_stream`` and the result is converted back to OpenAI chat
completion (streamed as SSE chunks).
"""

from __future__ import annotations

import json
import time
import uuid
from typing import AsyncIterator, Dict, List, Optional

import httpx
import jinja2

DEFAULT_CHAT_TEMPLATE = (
    "{% for m in messages %}<|start_header_id|>{{ m['role'] }}<|end_header_id|>\n\n{{ m['content'] }}<|eot_id|>"
    "{% endfor %}{% if add_generation_prompt %}<|start_header_id|>assistant<|end_header_id|>\n\n{% endif %}"
)


def models_response(models: List[Dict]) -> Dict:
    return {"object": "list", "data": [{"id": m["name"], "object": "model", "created": int(m.get("created", 0)),
                                        "owned_by": m.get("owner", "dstack")} for m in models]}


class OpenAIClient:
    def __init__(self, base_url: str, prefix: str = "/v1", client: Optional[httpx.AsyncClient] = None):
        self.url = base_url.rstrip("/") + prefix
        self.client = client or httpx.AsyncClient(timeout=600)

    async def generate(self, request: Dict) -> Dict:
        r = await self.client.post(self.url + "/chat/completions", json=request)
        r.raise_for_status()
        return r.json()

    async def stream(self, request: Dict) -> AsyncIterator[bytes]:
        async with self.client.stream("POST", self.url + "/chat/completions", json=request) as r:
            r.raise_for_status()
            async for chunk in r.aiter_bytes():
                yield chunk


class TGIClient:
    def __init__(self, base_url: str, chat_template: Optional[str] = None, eos_token: Optional[str] = None,
                 client: Optional[httpx.AsyncClient] = None):
        self.url = base_url.rstrip("/")
        env = jinja2.Environment(undefined=jinja2.StrictUndefined, trim_blocks=True, lstrip_blocks=True)
        env.globals["raise_exception"] = _raise
        self.template = env.from_string(chat_template or DEFAULT_CHAT_TEMPLATE)
        self.eos_token = eos_token or "<|eot_id|>"
        self.client = client or httpx.AsyncClient(timeout=600)

    def prompt(self, messages: List[Dict]) -> str:
        return self.template.render(messages=messages, add_generation_prompt=True, bos_token="", eos_token=self.eos_token)

    def _params(self, request: Dict) -> Dict:
        stop = request.get("stop") or []
        if isinstance(stop, str):
            stop = [stop]
        p = {"details": True, "decoder_input_details": False, "stop": stop + [self.eos_token]}
        if request.get("max_tokens"):
            p["max_new_tokens"] = request["max_tokens"]
        if request.get("temperature") is not None:
            t = request["temperature"]
            if t > 0:
                p["temperature"], p["do_sample"] = t, True
        if request.get("top_p") is not None and 0 < request["top_p"] < 1:
            p["top_p"] = request["top_p"]
        if request.get("seed") is not None:
            p["seed"] = request["seed"]
        return p

    async def generate(self, request: Dict) -> Dict:
        body = {"inputs": self.prompt(request["messages"]), "parameters": self._params(request)}
        r = await self.client.post(self.url + "/generate", json=body)
        r.raise_for_status()
        d = r.json()
        text = d.get("generated_text", "")
        for s in body["parameters"]["stop"]:
            if text.endswith(s):
                text = text[: -len(s)]
        det = d.get("details") or {}
        return {
            "id": f"chatcmpl-{uuid.uuid4().hex}", "object": "chat.completion", "created": int(time.time()),
            "model": request.get("model"),
            "choices": [{"index": 0, "message": {"role": "assistant", "content": text},
                         "finish_reason": "stop" if det.get("finish_reason") != "length" else "length"}],
            "usage": {"prompt_tokens": det.get("prefill_tokens", 0) if isinstance(det.get("prefill_tokens"), int) else 0,
                      "completion_tokens": det.get("generated_tokens", 0),
                      "total_tokens": det.get("generated_tokens", 0)},
        }

    async def stream(self, request: Dict) -> AsyncIterator[bytes]:
        body = {"inputs": self.prompt(request["messages"]), "parameters": self._params(request)}
        cid = f"chatcmpl-{uuid.uuid4().hex}"
        created = int(time.time())
        async with self.client.stream("POST", self.url + "/generate_stream", json=body) as r:
            r.raise_for_status()
            async for line in r.aiter_lines():
                if not line.startswith("data:"):
                    continue
                d = json.loads(line[5:])
                tok = (d.get("token") or {}).get("text", "")
                if tok in body["parameters"]["stop"]:
                    tok = ""
                finish = None
                if d.get("details"):
                    finish = "length" if d["details"].get("finish_reason") == "length" else "stop"
                chunk = {"id": cid, "object": "chat.completion.chunk", "created": created,
                         "model": request.get("model"),
                         "choices": [{"index": 0, "delta": {"content": tok} if tok else {}, "finish_reason": finish}]}
                yield f"data: {json.dumps(chunk)}\n\n".encode()
        yield b"data: [DONE]\n\n"


def _raise(msg):
    raise jinja2.exceptions.TemplateError(msg)


def make_client(model: Dict, base_url: str):
    if model.get("format") == "tgi":
        return TGIClient(base_url, model.get("chat_template"), model.get("eos_token"))
    return OpenAIClient(base_url, model.get("prefix", "/v1"))
