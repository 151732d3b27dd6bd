"""HOCON-subset parser (pyhocon / typesafe-config are not available).

Covers what the ytk-learn configs use (reference: ``config/model/*.conf``, parsed by
typesafe-config at ``J/worker/TrainWorker.java:142``):

* root object with or without braces; ``key : value``, ``key = value``, ``key { ... }``
* dotted keys (``a.b.c : 1``) create nested objects; repeated object keys MERGE,
  repeated non-object keys override (HOCON duplicate-key rule)
* values: double-quoted strings (JSON escapes), numbers (``1E-8``, ``-1``, ``5.28e-9``),
  ``true``/``false``/``yes``/``no``/``on``/``off``, ``null``, arrays, objects,
  unquoted strings (``???`` placeholders, ``gradient_boosting``)
* separators: commas and/or newlines; trailing commas allowed
* ``#`` and ``//`` comments (outside quoted strings)
* ``${path}`` substitutions resolved against the root after parsing

:class:`Config` wraps the tree with typed getters mirroring typesafe's
``getString/getInt/getDouble/getBoolean/getStringList/getDoubleList`` and
``withValue`` (the reference's programmatic overrides, ``TrainWorker.java:118-131``).
"""
from __future__ import annotations

import copy
import json
import re
from typing import Any, Dict, List, Optional

__all__ = ["parse", "parse_file", "Config", "ConfigError", "ConfigMissing", "PLACEHOLDER"]

PLACEHOLDER = "???"


class ConfigError(ValueError):
    pass


class ConfigMissing(ConfigError, KeyError):
    """Key absent (typesafe ``ConfigException.Missing``)."""


class _Subst:
    __slots__ = ("path", "optional")

    def __init__(self, path: str, optional: bool):
        self.path = path
        self.optional = optional


_NUM_RE = re.compile(r"^[+-]?(\d+\.?\d*|\.\d+)([eE][+-]?\d+)?$")
_UNQUOTED_STOP = set('{}[],:=#"\n') | {"\r"}


class _Parser:
    def __init__(self, text: str, origin: str = "<string>"):
        self.s = text
        self.i = 0
        self.n = len(text)
        self.origin = origin

    # ------------------------------------------------------------- lexing
    def err(self, msg):
        line = self.s.count("\n", 0, self.i) + 1
        raise ConfigError(f"{self.origin}:{line}: {msg}")

    def skip_ws(self, newlines=True):
        """Skip spaces, comments and (optionally) newlines. Returns True if a newline was seen."""
        saw_nl = False
        while self.i < self.n:
            c = self.s[self.i]
            if c == "\n":
                if not newlines:
                    return saw_nl
                saw_nl = True
                self.i += 1
            elif c in " \t\r﻿":
                self.i += 1
            elif c == "#" or self.s.startswith("//", self.i):
                j = self.s.find("\n", self.i)
                self.i = self.n if j < 0 else j
            else:
                break
        return saw_nl

    def peek(self):
        return self.s[self.i] if self.i < self.n else ""

    def quoted(self) -> str:
        if self.s.startswith('"""', self.i):
            j = self.s.find('"""', self.i + 3)
            if j < 0:
                self.err("unterminated triple-quoted string")
            out = self.s[self.i + 3:j]
            self.i = j + 3
            return out
        j = self.i + 1
        while j < self.n:
            c = self.s[j]
            if c == "\\":
                j += 2
                continue
            if c == '"':
                break
            if c == "\n":
                self.err("newline in quoted string")
            j += 1
        else:
            self.err("unterminated string")
        raw = self.s[self.i:j + 1]
        self.i = j + 1
        try:
            return json.loads(raw)
        except json.JSONDecodeError:
            self.err(f"bad string literal {raw!r}")

    # ------------------------------------------------------------- keys
    def key(self) -> List[str]:
        parts: List[str] = []
        cur = ""
        while self.i < self.n:
            c = self.peek()
            if c == '"':
                cur += self.quoted()
            elif c == ".":
                parts.append(cur.strip())
                cur = ""
                self.i += 1
            elif c in ":={" or c in " \t\r\n" or c == "#" or self.s.startswith("//", self.i) or c == "+":
                break
            elif c in '}],[':
                self.err(f"unexpected {c!r} in key")
            else:
                cur += c
                self.i += 1
        parts.append(cur.strip())
        if any(p == "" for p in parts):
            self.err("empty key")
        return parts

    # ------------------------------------------------------------- values
    def value(self) -> Any:
        self.skip_ws(newlines=True)
        c = self.peek()
        if c == "{":
            self.i += 1
            obj = self.object_body(closing="}")
            return obj
        if c == "[":
            self.i += 1
            return self.array_body()
        return self.simple_concat()

    def simple_concat(self) -> Any:
        """A scalar (possibly several unquoted/quoted pieces on one line joined by spaces)."""
        pieces: List[Any] = []
        quoted_any = False
        while self.i < self.n:
            c = self.peek()
            if c == '"':
                pieces.append(("q", self.quoted()))
                quoted_any = True
            elif self.s.startswith("${", self.i):
                j = self.s.find("}", self.i)
                if j < 0:
                    self.err("unterminated substitution")
                body = self.s[self.i + 2:j].strip()
                opt = body.startswith("?")
                pieces.append(("s", _Subst(body.lstrip("?").strip(), opt)))
                self.i = j + 1
            elif c in " \t":
                j = self.i
                while j < self.n and self.s[j] in " \t":
                    j += 1
                pieces.append(("w", self.s[self.i:j]))
                self.i = j
            elif c in _UNQUOTED_STOP or c in "}]" or self.s.startswith("//", self.i) or c == "":
                break
            else:
                j = self.i
                while j < self.n and self.s[j] not in _UNQUOTED_STOP and self.s[j] not in " \t}]$" \
                        and not self.s.startswith("//", j):
                    j += 1
                if j == self.i:  # lone '$'
                    j += 1
                pieces.append(("u", self.s[self.i:j]))
                self.i = j
        # strip leading / trailing whitespace pieces
        while pieces and pieces[0][0] == "w":
            pieces.pop(0)
        while pieces and pieces[-1][0] == "w":
            pieces.pop()
        if not pieces:
            self.err("expected a value")
        if len(pieces) == 1:
            kind, v = pieces[0]
            if kind == "q":
                return v
            if kind == "s":
                return v
            return _convert_unquoted(v)
        if any(k == "s" for k, _ in pieces):
            if len([p for p in pieces if p[0] != "w"]) == 1:
                return [p for p in pieces if p[0] == "s"][0][1]
            self.err("string concatenation with substitutions is not supported")
        return "".join(str(v) for _, v in pieces)

    def array_body(self) -> List[Any]:
        out: List[Any] = []
        while True:
            self.skip_ws()
            c = self.peek()
            if c == "]":
                self.i += 1
                return out
            if c == "":
                self.err("unterminated array")
            if c == ",":
                self.i += 1
                continue
            out.append(self.value())
            self.skip_ws(newlines=False)
            c = self.peek()
            if c == ",":
                self.i += 1
            elif c not in ("]", "\n", ""):
                self.skip_ws()
                if self.peek() != "]":
                    # newline separated elements handled by loop
                    pass

    def object_body(self, closing: Optional[str]) -> Dict[str, Any]:
        obj: Dict[str, Any] = {}
        while True:
            self.skip_ws()
            c = self.peek()
            if c == "":
                if closing is not None:
                    self.err("unterminated object")
                return obj
            if closing is not None and c == closing:
                self.i += 1
                return obj
            if c == ",":
                self.i += 1
                continue
            path = self.key()
            self.skip_ws(newlines=False)
            c = self.peek()
            append = False
            if c in ":=":
                self.i += 1
            elif self.s.startswith("+=", self.i):
                self.i += 2
                append = True
            elif c != "{":
                self.err(f"expected ':' '=' or '{{' after key {'.'.join(path)!r}")
            v = self.value()
            _assign(obj, path, v, append)
            self.skip_ws(newlines=False)
            c = self.peek()
            if c == ",":
                self.i += 1


def _convert_unquoted(tok: str) -> Any:
    t = tok.strip()
    low = t.lower()
    if low in ("true", "yes", "on"):
        return True
    if low in ("false", "no", "off"):
        return False
    if low == "null":
        return None
    if _NUM_RE.match(t):
        if re.match(r"^[+-]?\d+$", t):
            return int(t)
        return float(t)
    return t


def _merge(a: Any, b: Any) -> Any:
    if isinstance(a, dict) and isinstance(b, dict):
        out = dict(a)
        for k, v in b.items():
            out[k] = _merge(out[k], v) if k in out else v
        return out
    return b


def _assign(obj: Dict[str, Any], path: List[str], v: Any, append: bool = False):
    cur = obj
    for p in path[:-1]:
        nxt = cur.get(p)
        if not isinstance(nxt, dict):
            nxt = {}
            cur[p] = nxt
        cur = nxt
    last = path[-1]
    if append:
        prev = cur.get(last, [])
        if not isinstance(prev, list):
            raise ConfigError(f"+= on non-array key {'.'.join(path)}")
        cur[last] = prev + [v]
    elif last in cur:
        cur[last] = _merge(cur[last], v)
    else:
        cur[last] = v


def _lookup(root: Dict[str, Any], path: str):
    cur: Any = root
    for p in _split_path(path):
        if not isinstance(cur, dict) or p not in cur:
            raise ConfigMissing(path)
        cur = cur[p]
    return cur


def _split_path(path: str) -> List[str]:
    out, cur, i = [], "", 0
    while i < len(path):
        c = path[i]
        if c == '"':
            j = path.index('"', i + 1)
            cur += path[i + 1:j]
            i = j + 1
            continue
        if c == ".":
            out.append(cur)
            cur = ""
        else:
            cur += c
        i += 1
    out.append(cur)
    return out


def _resolve(node: Any, root: Dict[str, Any], depth=0):
    if depth > 64:
        raise ConfigError("substitution cycle")
    if isinstance(node, dict):
        for k in list(node.keys()):
            v = _resolve(node[k], root, depth)
            if v is _DROP:
                del node[k]
            else:
                node[k] = v
        return node
    if isinstance(node, list):
        return [x for x in (_resolve(v, root, depth) for v in node) if x is not _DROP]
    if isinstance(node, _Subst):
        try:
            return _resolve(copy.deepcopy(_lookup(root, node.path)), root, depth + 1)
        except ConfigMissing:
            import os
            if node.path in os.environ:
                return os.environ[node.path]
            if node.optional:
                return _DROP
            raise ConfigError(f"unresolved substitution ${{{node.path}}}")
    return node


_DROP = object()


def parse(text: str, origin: str = "<string>") -> "Config":
    p = _Parser(text, origin)
    p.skip_ws()
    if p.peek() == "{":
        p.i += 1
        root = p.object_body(closing="}")
        p.skip_ws()
        if p.i < p.n:
            p.err("trailing content after root object")
    else:
        root = p.object_body(closing=None)
    root = _resolve(root, root)
    return Config(root)


def parse_file(path: str) -> "Config":
    with open(path, "r", encoding="utf-8") as f:
        return parse(f.read(), origin=path)


# ---------------------------------------------------------------------------
class Config:
    """Immutable-ish view over a parsed tree with typesafe-style typed getters."""

    def __init__(self, root: Optional[Dict[str, Any]] = None):
        self.root = root if root is not None else {}

    # generic
    def has(self, path: str) -> bool:
        try:
            _lookup(self.root, path)
            return True
        except ConfigMissing:
            return False

    def get(self, path: str, default: Any = ConfigMissing) -> Any:
        try:
            return _lookup(self.root, path)
        except ConfigMissing:
            if default is ConfigMissing:
                raise
            return default

    def _typed(self, path, default, conv, tname):
        try:
            v = _lookup(self.root, path)
        except ConfigMissing:
            if default is ConfigMissing:
                raise
            return default
        if v == PLACEHOLDER:
            raise ConfigError(f"config key {path} is a required placeholder (???); set it")
        try:
            return conv(v)
        except (TypeError, ValueError):
            raise ConfigError(f"config key {path}: expected {tname}, got {v!r}")

    def get_string(self, path, default=ConfigMissing) -> str:
        def conv(v):
            if isinstance(v, (dict, list)):
                raise TypeError
            if isinstance(v, bool):
                return "true" if v else "false"
            if v is None:
                raise TypeError
            return str(v)
        return self._typed(path, default, conv, "string")

    def get_int(self, path, default=ConfigMissing) -> int:
        def conv(v):
            if isinstance(v, bool):
                raise TypeError
            if isinstance(v, str):
                v = _convert_unquoted(v)
            f = float(v)
            if f != int(f):
                raise ValueError
            return int(f)
        return self._typed(path, default, conv, "int")

    def get_double(self, path, default=ConfigMissing) -> float:
        def conv(v):
            if isinstance(v, bool):
                raise TypeError
            return float(v)
        return self._typed(path, default, conv, "number")

    get_float = get_double

    def get_bool(self, path, default=ConfigMissing) -> bool:
        def conv(v):
            if isinstance(v, bool):
                return v
            if isinstance(v, str) and v.lower() in ("true", "yes", "on", "false", "no", "off"):
                return v.lower() in ("true", "yes", "on")
            raise TypeError
        return self._typed(path, default, conv, "boolean")

    def get_list(self, path, default=ConfigMissing) -> list:
        def conv(v):
            if not isinstance(v, list):
                raise TypeError
            return list(v)
        return self._typed(path, default, conv, "list")

    def get_string_list(self, path, default=ConfigMissing) -> List[str]:
        return [str(x) for x in self.get_list(path, default)]

    def get_double_list(self, path, default=ConfigMissing) -> List[float]:
        return [float(x) for x in self.get_list(path, default)]

    def get_int_list(self, path, default=ConfigMissing) -> List[int]:
        return [int(x) for x in self.get_list(path, default)]

    def get_config(self, path) -> "Config":
        v = self.get(path)
        if not isinstance(v, dict):
            raise ConfigError(f"config key {path} is not an object")
        return Config(v)

    # overrides (typesafe withValue)
    def with_value(self, path: str, value: Any) -> "Config":
        root = copy.deepcopy(self.root)
        cur = root
        parts = _split_path(path)
        for p in parts[:-1]:
            if not isinstance(cur.get(p), dict):
                cur[p] = {}
            cur = cur[p]
        cur[parts[-1]] = copy.deepcopy(value)
        return Config(root)

    def with_overrides(self, overrides: Dict[str, Any]) -> "Config":
        c = self
        for k, v in overrides.items():
            c = c.with_value(k, v)
        return c

    def flatten(self, prefix: str = "") -> Dict[str, Any]:
        out: Dict[str, Any] = {}

        def rec(node, pre):
            for k, v in node.items():
                key = f"{pre}{k}"
                if isinstance(v, dict):
                    rec(v, key + ".")
                else:
                    out[key] = v
        rec(self.root, prefix)
        return out

    def to_dict(self) -> Dict[str, Any]:
        return copy.deepcopy(self.root)

    def __repr__(self):
        return f"Config({self.root!r})"


def parse_override_value(text: str) -> Any:
    """Parse a CLI override value (``key=value``) with HOCON scalar/array rules."""
    c = parse(f"v : {text}")
    return c.get("v")
