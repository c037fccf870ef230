"""Minimal KDL document parser for FleetFlow's ``fleet.kdl`` files.

The reference parses with the third-party ``kdl = "6"`` crate (workspace
Cargo.toml; no Cargo.lock, so the exact version is unpinned).  That crate
implements KDL 2.0 and falls back to KDL 1.0 when a document is not valid
v2.  This module implements the grammar FleetFlow files use, following the
published KDL 2.0 specification:

* nodes: ``name entry* children? terminator``; a name is a bare identifier or a
  quoted string; ``(type)`` annotations are accepted and dropped;
* entries: arguments and ``key=value`` properties, kept in source order (the
  reference reads ``entries().first()`` and ``get(key)``; ``get`` returns the
  rightmost property of that name);
* values: quoted strings with escapes (``\\n \\t \\" \\\\ \\b \\f \\s \\/ \\u{..}``,
  whitespace escapes), multi-line ``\"\"\"`` strings with dedent, raw strings
  (``#"..."#``; v1 ``r"..."``/``r#"..."#``), bare identifier strings, numbers
  (decimal with ``_``, exponents, ``0x``/``0o``/``0b``), the keywords ``#true``,
  ``#false``, ``#null``, ``#inf``, ``#-inf``, ``#nan``;
* the KDL 1 keywords ``true``/``false``/``null`` as bare values (the crate's v1
  fallback; ``examples/hello-world/flow.kdl:19`` writes ``read_only=true``);
* comments ``//``, nested ``/* */`` and slashdash ``/-`` on nodes, entries and
  children blocks; ``;`` terminators; ``\\`` line continuations.

Values map to Python ``str``/``int``/``float``/``bool``/``None``.
"""
from __future__ import annotations

from dataclasses import dataclass, field

_NEWLINES = "\n\r\x0b\x0c\x85\u2028\u2029"
_SPACES = " \t\ufeff\u00a0\u1680\u2000\u2001\u2002\u2003\u2004\u2005\u2006\u2007\u2008\u2009\u200a\u202f\u205f\u3000"
_NON_IDENT = set('\\/(){};[]="#') | set(_NEWLINES) | set(_SPACES)


class KdlError(ValueError):
    pass


@dataclass
class KdlNode:
    name: str
    entries: list = field(default_factory=list)  # [(key or None, value)]
    children: list | None = None                 # None = no children block

    def args(self):
        return [v for k, v in self.entries if k is None]

    def get(self, key):
        """Rightmost property ``key`` (None if absent)."""
        for k, v in reversed(self.entries):
            if k == key:
                return v
        return None

    def has(self, key):
        return any(k == key for k, _ in self.entries)

    def first(self):
        """Value of the first entry, argument or property (``entries().first()``)."""
        return self.entries[0][1] if self.entries else None


def is_str(v):
    return isinstance(v, str)


def is_int(v):
    return isinstance(v, int) and not isinstance(v, bool)


def as_str(v):
    return v if isinstance(v, str) else None


def as_int(v):
    return v if is_int(v) else None


class _Parser:
    def __init__(self, text: str):
        self.s = text
        self.i = 0
        self.n = len(text)

    # -- low level -------------------------------------------------------------
    def err(self, msg):
        line = self.s.count("\n", 0, self.i) + 1
        col = self.i - (self.s.rfind("\n", 0, self.i) + 1) + 1
        raise KdlError(f"KDL parse error at {line}:{col}: {msg}")

    def peek(self, k=0):
        j = self.i + k
        return self.s[j] if j < self.n else ""

    def startswith(self, t):
        return self.s.startswith(t, self.i)

    def skip_block_comment(self):
        # at "/*"; comments nest
        depth = 0
        while self.i < self.n:
            if self.startswith("/*"):
                depth += 1
                self.i += 2
            elif self.startswith("*/"):
                depth -= 1
                self.i += 2
                if depth == 0:
                    return
            else:
                self.i += 1
        self.err("unterminated block comment")

    def skip_line_comment(self):
        while self.i < self.n and self.s[self.i] not in _NEWLINES:
            self.i += 1

    def skip_ws(self):
        """Inline whitespace, block comments and line continuations (node-space)."""
        while self.i < self.n:
            c = self.s[self.i]
            if c in _SPACES:
                self.i += 1
            elif self.startswith("/*"):
                self.skip_block_comment()
            elif c == "\\":
                # line continuation: "\" ws* (line-comment)? newline
                j = self.i + 1
                while j < self.n and self.s[j] in _SPACES:
                    j += 1
                if self.s.startswith("//", j):
                    while j < self.n and self.s[j] not in _NEWLINES:
                        j += 1
                if j < self.n and self.s[j] in _NEWLINES:
                    j += 2 if self.s.startswith("\r\n", j) else 1
                    self.i = j
                elif j >= self.n:
                    self.i = j
                else:
                    return
            else:
                return

    def skip_line_space(self):
        """Whitespace, newlines and all comments between nodes."""
        while self.i < self.n:
            c = self.s[self.i]
            if c in _SPACES or c in _NEWLINES:
                self.i += 1
            elif self.startswith("//"):
                self.skip_line_comment()
            elif self.startswith("/*"):
                self.skip_block_comment()
            else:
                return

    # -- values ------------------------------------------------------------------
    def ident(self):
        j = self.i
        while j < self.n and self.s[j] not in _NON_IDENT:
            j += 1
        if j == self.i:
            self.err(f"unexpected character {self.peek()!r}")
        t = self.s[self.i:j]
        self.i = j
        return t

    def quoted(self):
        if self.startswith('"""'):
            return self.multiline()
        self.i += 1
        out = []
        while True:
            if self.i >= self.n:
                self.err("unterminated string")
            c = self.s[self.i]
            if c == '"':
                self.i += 1
                return "".join(out)
            if c == "\\":
                out.append(self.escape())
                continue
            if c in "\r\n":
                self.err("newline in single-line string")
            out.append(c)
            self.i += 1

    def escape(self):
        # at "\"
        self.i += 1
        c = self.peek()
        simple = {"n": "\n", "r": "\r", "t": "\t", "\\": "\\", '"': '"', "b": "\b", "f": "\f", "s": " ",
                  "/": "/"}
        if c in simple:
            self.i += 1
            return simple[c]
        if c == "u":
            if self.peek(1) != "{":
                self.err("bad unicode escape")
            j = self.s.find("}", self.i)
            if j < 0:
                self.err("bad unicode escape")
            try:
                ch = chr(int(self.s[self.i + 2:j], 16))
            except ValueError:
                self.err("bad unicode escape")
            self.i = j + 1
            return ch
        if c and (c in _SPACES or c in _NEWLINES):
            while self.i < self.n and (self.s[self.i] in _SPACES or self.s[self.i] in _NEWLINES):
                self.i += 1
            return ""
        self.err(f"bad escape \\{c}")

    def multiline(self):
        # at '"""' followed by a newline; body lines dedented by the closing line's prefix
        self.i += 3
        if self.startswith("\r\n"):
            self.i += 2
        elif self.peek() in _NEWLINES and self.peek():
            self.i += 1
        else:
            self.err('multi-line string must start with a newline after """')
        out = []
        while True:
            if self.i >= self.n:
                self.err("unterminated multi-line string")
            if self.startswith('"""'):
                self.i += 3
                break
            c = self.s[self.i]
            if c == "\\":
                out.append(self.escape())
                continue
            out.append(c)
            self.i += 1
        body = "".join(out).replace("\r\n", "\n")
        lines = body.split("\n")
        prefix = lines[-1]
        if prefix.strip(" \t"):
            self.err("closing \"\"\" must be on its own line")
        res = []
        for ln in lines[:-1]:
            if not ln.strip(" \t"):
                res.append("")
            elif ln.startswith(prefix):
                res.append(ln[len(prefix):])
            else:
                self.err("inconsistent multi-line string indentation")
        return "\n".join(res)

    def raw(self):
        # at '#'+ '"' (v2) or 'r' '#'* '"' (v1)
        if self.peek() == "r":
            self.i += 1
        h = 0
        while self.peek() == "#":
            h += 1
            self.i += 1
        if self.peek() != '"':
            self.err("bad raw string")
        multi = self.startswith('"""')
        self.i += 3 if multi else 1
        close = ('"""' if multi else '"') + "#" * h
        j = self.s.find(close, self.i)
        if j < 0:
            self.err("unterminated raw string")
        body = self.s[self.i:j]
        self.i = j + len(close)
        if multi:
            body = body.replace("\r\n", "\n")
            if body.startswith("\n"):
                body = body[1:]
            lines = body.split("\n")
            prefix = lines[-1]
            body = "\n".join(ln[len(prefix):] if ln.startswith(prefix) else ln.strip(" \t") for ln in lines[:-1])
        return body

    def number(self, tok):
        t = tok.replace("_", "")
        sign = 1
        body = t
        if body[:1] in "+-":
            sign = -1 if body[0] == "-" else 1
            body = body[1:]
        try:
            if body[:2] in ("0x", "0X"):
                return sign * int(body[2:], 16)
            if body[:2] in ("0o", "0O"):
                return sign * int(body[2:], 8)
            if body[:2] in ("0b", "0B"):
                return sign * int(body[2:], 2)
            if any(ch in body for ch in ".eE"):
                return sign * float(body)
            return sign * int(body, 10)
        except ValueError:
            self.err(f"bad number {tok!r}")

    def value(self):
        """One value; returns (kind, v) where kind is 'str' for strings that may
        be a property key, else 'val'."""
        c = self.peek()
        if c == "(":  # type annotation
            self.type_annotation()
            c = self.peek()
        if c == '"':
            return "str", self.quoted()
        if c == "#":
            if self.peek(1) == '"' or self.peek(1) == "#":
                return "val", self.raw()
            tok = self.ident_after_hash()
            kw = {"true": True, "false": False, "null": None, "inf": float("inf"), "-inf": float("-inf"),
                  "nan": float("nan")}
            if tok not in kw:
                self.err(f"unknown keyword #{tok}")
            return "val", kw[tok]
        if c == "r" and (self.peek(1) == '"' or (self.peek(1) == "#" and self._raw_v1_ahead())):
            return "val", self.raw()
        tok = self.ident()
        if tok[0].isdigit() or (tok[0] in "+-." and len(tok) > 1 and (tok[1].isdigit() or tok[1] == ".")):
            return "val", self.number(tok)
        if tok in ("true", "false", "null"):  # KDL 1 keywords (v1 fallback)
            return "val", {"true": True, "false": False, "null": None}[tok]
        return "str", tok

    def _raw_v1_ahead(self):
        j = self.i + 1
        while j < self.n and self.s[j] == "#":
            j += 1
        return j < self.n and self.s[j] == '"'

    def ident_after_hash(self):
        self.i += 1
        return self.ident()

    def type_annotation(self):
        self.i += 1
        self.skip_ws()
        if self.peek() == '"':
            self.quoted()
        else:
            self.ident()
        self.skip_ws()
        if self.peek() != ")":
            self.err("unterminated type annotation")
        self.i += 1
        self.skip_ws()

    # -- structure ---------------------------------------------------------------
    def document(self, top=True):
        nodes = []
        while True:
            self.skip_line_space()
            if self.i >= self.n:
                if not top:
                    self.err("missing '}'")
                return nodes
            if self.peek() == "}":
                if top:
                    self.err("unexpected '}'")
                return nodes
            if self.peek() == ";":
                self.i += 1
                continue
            slashdash = False
            if self.startswith("/-"):
                self.i += 2
                slashdash = True
                self.skip_line_space()
            node = self.node()
            if not slashdash:
                nodes.append(node)

    def node(self):
        if self.peek() == "(":
            self.type_annotation()
        if self.peek() == '"':
            name = self.quoted()
        elif self.peek() == "#" or (self.peek() == "r" and self._raw_v1_ahead()):
            name = self.raw()
        else:
            name = self.ident()
        node = KdlNode(name)
        while True:
            before = self.i
            self.skip_ws()
            c = self.peek()
            if c == "" or c in _NEWLINES or c == ";":
                if c == ";":
                    self.i += 1
                return node
            if self.startswith("//"):
                self.skip_line_comment()
                return node
            if c == "}":
                return node
            slashdash = False
            if self.startswith("/-"):
                self.i += 2
                slashdash = True
                self.skip_line_space()
                c = self.peek()
            if c == "{":
                self.i += 1
                kids = self.document(top=False)
                self.i += 1  # '}'
                if not slashdash:
                    if node.children is not None:
                        self.err("a node has at most one children block")
                    node.children = kids
                continue
            if node.children is not None and not slashdash:
                self.err("entries after a children block")
            if self.i == before and not slashdash:
                self.err("missing whitespace between entries")
            kind, v = self.value()
            if kind == "str" and self.peek() == "=":
                self.i += 1
                self.skip_ws()
                _, pv = self.value()
                if not slashdash:
                    node.entries.append((v, pv))
            elif not slashdash:
                node.entries.append((None, v))


def parse(text: str) -> list[KdlNode]:
    """Parse a KDL document into its top-level nodes."""
    return _Parser(text).document()


def _fmt_value(v):
    if v is True:
        return "#true"
    if v is False:
        return "#false"
    if v is None:
        return "#null"
    if isinstance(v, str):
        return '"' + v.replace("\\", "\\\\").replace('"', '\\"').replace("\n", "\\n").replace("\t", "\\t") + '"'
    return repr(v)


def dumps(nodes: list[KdlNode], indent: int = 0) -> str:
    """Serialise nodes back to KDL 2 text (used to re-emit included files)."""
    out = []
    pad = "    " * indent
    for nd in nodes:
        parts = [_fmt_value(nd.name)]
        for k, v in nd.entries:
            parts.append(_fmt_value(v) if k is None else f"{_fmt_value(k)}={_fmt_value(v)}")
        line = pad + " ".join(parts)
        if nd.children is not None:
            line += " {\n" + dumps(nd.children, indent + 1) + pad + "}"
        out.append(line + "\n")
    return "".join(out)
