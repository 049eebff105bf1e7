"""The reply envelope and request validation of the reference service, reproduced exactly.

`NATSResponse{ok, error,omitempty, data,omitempty}` (`/root/reference/nats_llm_studio.go:186-190`):
* success: {"ok":true,"data":{...}} (no "error" key);
* validation errors use respondError(msg, err, nil): the nil map inside interface{} is
  not omitted by Go's omitempty, so the wire form carries "data":null;
* marshalling failure: the literal fallback (`:211`).
Go's encoding/json escapes <, >, & as \\u003c etc.; any JSON-equivalent output parses the same.
"""
from __future__ import annotations

import json
from typing import Any, Optional

FALLBACK = b'{"ok":false,"error":"internal error serializing response"}'
_NO_DATA = object()
ANON_CHAT_STRUCT = 'struct { Model string "json:\\"model\\"" }'


def _go_json(obj: Any) -> bytes:
    s = json.dumps(obj, ensure_ascii=False, separators=(",", ":"), allow_nan=False)
    s = s.replace("<", "\\u003c").replace(">", "\\u003e").replace("&", "\\u0026")
    return s.encode("utf-8")


def ok(data: Any) -> bytes:
    try:
        return _go_json({"ok": True, "data": data})
    except (TypeError, ValueError):
        return FALLBACK


def error(err: str, data: Any = None) -> bytes:
    """respondError(msg, err, extraData): data=None -> "data":null (Go nil map in interface{})."""
    try:
        return _go_json({"ok": False, "error": err, "data": data})
    except (TypeError, ValueError):
        return FALLBACK


def failure(err: str, data: Any) -> bytes:
    """NATSResponse{OK:false, Error, Data} built directly (pull/delete failure paths)."""
    return error(err, data)


# ---------------------------------------------------------------------------
# Go encoding/json error texts for the JSON probes of the handlers
# ---------------------------------------------------------------------------

def go_json_error(raw: bytes, struct: str = "", fields: Optional[dict] = None) -> Optional[str]:
    """Return Go's json.Unmarshal error text for `raw` decoded into a struct with string
    `fields` ({json_name: GoFieldName}), or None if it decodes fine."""
    try:
        text = raw.decode("utf-8")
    except UnicodeDecodeError:
        return "invalid character '\\ufffd' looking for beginning of value"
    if not text.strip():
        return "unexpected end of JSON input"
    try:
        obj = json.loads(text)
    except json.JSONDecodeError as e:
        if e.pos >= len(text.rstrip()):
            return "unexpected end of JSON input"
        ch = text[e.pos]
        if e.msg.startswith("Expecting value"):
            return f"invalid character '{ch}' looking for beginning of value"
        if e.msg.startswith("Expecting property name"):
            return f"invalid character '{ch}' looking for beginning of object key string"
        if e.msg.startswith("Expecting ':'"):
            return f"invalid character '{ch}' after object key"
        if e.msg.startswith("Expecting ',' delimiter"):
            return f"invalid character '{ch}' after object key:value pair"
        if e.msg.startswith("Extra data"):
            return f"invalid character '{ch}' after top-level value"
        return f"invalid character '{ch}' looking for beginning of value"
    if fields and isinstance(obj, dict):
        gotype = {bool: "bool", int: "number", float: "number", list: "array", dict: "object"}
        for k, v in obj.items():
            for jn, fn in fields.items():
                if k.lower() == jn.lower() and v is not None and not isinstance(v, str):
                    t = gotype.get(type(v), "value")
                    return f"json: cannot unmarshal {t} into Go struct field {struct}.{jn} of type string"
    if not isinstance(obj, dict) and obj is not None:
        t = {bool: "bool", int: "number", float: "number", list: "array", str: "string"}.get(type(obj), "value")
        tname = ("nats_llm_studio." + struct) if struct else ANON_CHAT_STRUCT
        return f"json: cannot unmarshal {t} into Go value of type {tname}"
    return None


def get_field(raw: bytes, name: str) -> str:
    """Go's case-insensitive struct-field match for a string field ('' when absent/null)."""
    obj = json.loads(raw.decode("utf-8"))
    if not isinstance(obj, dict):
        return ""
    if name in obj:
        v = obj[name]
    else:
        v = next((vv for k, vv in obj.items() if k.lower() == name.lower()), "")
    return v if isinstance(v, str) else ""
