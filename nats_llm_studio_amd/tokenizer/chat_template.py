"""Chat templating from GGUF `tokenizer.chat_template` (jinja2, sandboxed)."""
from __future__ import annotations

from typing import Dict, List, Optional

import jinja2
from jinja2.sandbox import ImmutableSandboxedEnvironment

from .synthetic import GRANITE_TEMPLATE, LLAMA3_TEMPLATE, MISTRAL_TEMPLATE

_ENV = ImmutableSandboxedEnvironment(trim_blocks=True, lstrip_blocks=True, undefined=jinja2.Undefined)


def _raise(msg):
    raise jinja2.exceptions.TemplateError(msg)


_ENV.globals["raise_exception"] = _raise


def default_template(arch: str, tok_model: str) -> str:
    if arch == "granite":
        return GRANITE_TEMPLATE
    if tok_model == "llama":
        return MISTRAL_TEMPLATE
    return LLAMA3_TEMPLATE


def _content_text(content) -> str:
    if isinstance(content, str):
        return content
    if isinstance(content, list):   # OpenAI multi-part content: keep text parts
        return "".join(p.get("text", "") for p in content if isinstance(p, dict))
    return "" if content is None else str(content)


class ChatTemplate:
    def __init__(self, source: str, bos_token: str = "", eos_token: str = ""):
        self.source = source
        self.template = _ENV.from_string(source)
        self.bos_token = bos_token
        self.eos_token = eos_token

    def render(self, messages: List[Dict], add_generation_prompt: bool = True, tools: Optional[list] = None) -> str:
        msgs = [{**m, "content": _content_text(m.get("content"))} for m in messages]
        return self.template.render(messages=msgs, add_generation_prompt=add_generation_prompt,
                                    bos_token=self.bos_token, eos_token=self.eos_token, tools=tools)
