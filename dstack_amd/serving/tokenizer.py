"""Tokenizers for the serving engine.

* ``HFTokenizer``: a checkpoint's ``tokenizer.json`` through the ``tokenizers`` library, with the
  chat template from ``tokenizer_config.json`` (Jinja) when present.
* ``ByteTokenizer``: UTF-8 bytes as token ids (offset by the special ids) for built-in
  random-weight configs — there is no network to fetch a vocabulary, and a random model's outputs
  carry no meaning anyway; it keeps the OpenAI API path (text in, text out, token counts) whole.

Both expose ``encode``, ``decode``, ``apply_chat_template``, ``eos_token_ids`` and ``bos_token_id``.
"""

from __future__ import annotations

import json
import os


def _llama3_chat(messages, add_generation_prompt=True) -> str:
    """The Llama-3 instruct chat format (used when a checkpoint ships no template)."""
    out = "<|begin_of_text|>"
    for m in messages:
        out += f"<|start_header_id|>{m['role']}<|end_header_id|>\n\n{_content(m)}<|eot_id|>"
    if add_generation_prompt:
        out += "<|start_header_id|>assistant<|end_header_id|>\n\n"
    return out


def _content(m) -> str:
    c = m.get("content", "")
    if isinstance(c, list):  # OpenAI content parts
        return "".join(p.get("text", "") for p in c if isinstance(p, dict))
    return c or ""


class ByteTokenizer:
    PAD, BOS, EOS = 0, 1, 2
    OFFSET = 3

    def __init__(self, vocab_size: int):
        self.vocab_size = vocab_size
        self.bos_token_id = self.BOS
        self.eos_token_ids = (self.EOS,)

    def encode(self, text: str, add_bos: bool = True) -> list[int]:
        ids = [b + self.OFFSET for b in text.encode("utf-8")]
        return ([self.BOS] if add_bos else []) + ids

    def decode(self, ids) -> str:
        # ids outside the byte range (a random model samples the whole vocabulary) map onto bytes
        bs = bytes((i - self.OFFSET) % 256 for i in ids if i >= self.OFFSET)
        return bs.decode("utf-8", errors="replace")

    def apply_chat_template(self, messages, add_generation_prompt=True) -> str:
        out = ""
        for m in messages:
            out += f"<{m['role']}>{_content(m)}\n"
        return out + ("<assistant>" if add_generation_prompt else "")


class HFTokenizer:
    def __init__(self, path: str):
        from tokenizers import Tokenizer

        self.tok = Tokenizer.from_file(os.path.join(path, "tokenizer.json"))
        self.vocab_size = self.tok.get_vocab_size()
        cfg = {}
        p = os.path.join(path, "tokenizer_config.json")
        if os.path.exists(p):
            with open(p) as f:
                cfg = json.load(f)
        self.chat_template = cfg.get("chat_template")
        self.bos_token_id = self._id(cfg.get("bos_token"))
        eos = [self._id(cfg.get("eos_token"))]
        for extra in ("<|eot_id|>", "<|end_of_text|>"):
            eos.append(self.tok.token_to_id(extra))
        self.eos_token_ids = tuple(sorted({e for e in eos if e is not None}))
        self._bos_text = cfg.get("bos_token") if isinstance(cfg.get("bos_token"), str) else None

    def _id(self, tok):
        if isinstance(tok, dict):
            tok = tok.get("content")
        return self.tok.token_to_id(tok) if isinstance(tok, str) else None

    def encode(self, text: str, add_bos: bool = True) -> list[int]:
        ids = self.tok.encode(text, add_special_tokens=False).ids
        if add_bos and self.bos_token_id is not None and (not ids or ids[0] != self.bos_token_id):
            ids = [self.bos_token_id] + ids
        return ids

    def decode(self, ids) -> str:
        return self.tok.decode(list(ids), skip_special_tokens=True)

    def apply_chat_template(self, messages, add_generation_prompt=True) -> str:
        if not self.chat_template:
            return _llama3_chat(messages, add_generation_prompt)
        import jinja2

        env = jinja2.Environment(trim_blocks=True, lstrip_blocks=True)
        env.globals["raise_exception"] = lambda msg: (_ for _ in ()).throw(ValueError(msg))
        return env.from_string(self.chat_template).render(
            messages=messages, add_generation_prompt=add_generation_prompt, bos_token=self._bos_text or "")


def load_tokenizer(model_path: str | None, vocab_size: int):
    if model_path and os.path.exists(os.path.join(model_path, "tokenizer.json")):
        return HFTokenizer(model_path)
    return ByteTokenizer(vocab_size)
