#!/usr/bin/env python3
"""go_cgo_check.py — a static check of the reference-side cgo binding without a Go toolchain.

The image has no `go`, so `tendermint-fork_amd/go/tmedgpu/tmedgpu.go` and the Go snippets of
INTEGRATION.md are never compiled here.  Round 5 broke the package that way (`batchArgs(&a, ...)`
with `a` already an `*arena`).  This tool parses the Go text with a small Go parser (tokens with
semicolon insertion, statements, expressions, types), infers the types of the expressions it can,
and checks them against the C header as clang reads it (`clang -Xclang -ast-dump=json`) and
against the package's own declarations:

  C1  every `C.f(...)` names a prototype of include/tmed25519.h (or cgo's malloc/free/GoString)
      with the same argument count, and every argument whose type is known has the cgo type of
      that parameter (`*C.uint8_t` for `const uint8_t *`, `**C.tmed_ctx` for `tmed_ctx **`, ...);
  C2  every field of a `C.tmed_x{...}` literal and every `.field` read or written on a C struct
      exists in that typedef, and a value of known type assigned to it has the field's cgo type;
  C3  every `C.TMED_*` constant is a macro of the header;
  C4  every call of a package function, method or func-typed variable passes the declared number
      of arguments, each of the declared type where both are known (pointer depth included:
      `*arena` vs `**arena`), and every field of a package struct literal / selector exists;
  C5  (package `types`) every `tmedgpu.X` is an exported name of the package,
      every method / field used on a tmedgpu type exists and is exported, calls pass the declared
      number of arguments, and a pointer result that comes with an error (`p, err := f()`) is not
      dereferenced on a path where err may be non-nil.

Types it cannot infer (the reference's own types in the snippets, untyped constants) are skipped,
never guessed.  Usage: python tools/go_cgo_check.py  (exit 1 and one line per finding).
Test: tests/test_go_binding.py (also feeds it the round-5 text to show it fails on it).
"""
from __future__ import annotations

import json
import os
import re
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GO_FILE = os.path.join(ROOT, "tendermint-fork_amd", "go", "tmedgpu", "tmedgpu.go")
HEADER = os.path.join(ROOT, "include", "tmed25519.h")
INTEGRATION = os.path.join(ROOT, "INTEGRATION.md")


# ----------------------------------------------------------------------------------- C header

def _clang():
    for c in ("/opt/rocm/lib/llvm/bin/clang", shutil.which("clang") or ""):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("go_cgo_check: clang not found (needed to read the C header)")


def c_to_go(qt: str) -> str:
    """cgo's Go type for a C type as clang prints it ('const uint8_t *' -> '*C.uint8_t')."""
    t = qt.replace("const", " ").strip()
    t = re.sub(r"\s+", " ", t)
    m = re.match(r"^(.*?)\s*\[(\d+)\]$", t)
    if m:
        return "[%s]%s" % (m.group(2), c_to_go(m.group(1)))
    if t.endswith("*"):
        inner = t[:-1].strip()
        if inner == "void":
            return "unsafe.Pointer"
        return "*" + c_to_go(inner)
    if t == "void":
        return ""
    if t.startswith("struct "):
        t = "struct_" + t[len("struct "):]
    return "C." + t.replace(" ", "")


class Header:
    """Prototypes, typedef'd structs and macros of the C header."""

    def __init__(self, path: str = HEADER, text: str | None = None):
        clang = _clang()
        src = ["-x", "c", "-"] if text is not None else [path]
        inc = ["-I", os.path.dirname(path)]
        ast = subprocess.run([clang, "-Xclang", "-ast-dump=json", "-fsyntax-only"] + inc + src,
                             input=text, capture_output=True, text=True, check=True).stdout
        mac = subprocess.run([clang, "-E", "-dM"] + inc + src, input=text, capture_output=True, text=True,
                             check=True).stdout
        self.funcs: dict[str, tuple[list[str], str]] = {}   # name -> ([param go types], go result)
        self.structs: dict[str, dict[str, str]] = {}        # typedef name -> {field: go type}
        self.macros = set(re.findall(r"^#define\s+(\w+)", mac, re.M))
        records: dict[str, dict[str, str]] = {}
        for d in json.loads(ast).get("inner", []):
            k = d.get("kind")
            if k == "FunctionDecl":
                params = [c_to_go(p["type"]["qualType"]) for p in d.get("inner", []) if p.get("kind") == "ParmVarDecl"]
                res = d["type"]["qualType"].split("(")[0].strip()
                self.funcs[d["name"]] = (params, c_to_go(res))
            elif k == "RecordDecl" and d.get("completeDefinition"):
                records[d["id"]] = {f["name"]: c_to_go(f["type"]["qualType"]) for f in d.get("inner", [])
                                    if f.get("kind") == "FieldDecl"}
            elif k == "TypedefDecl":
                inner = d.get("inner", [{}])[0]
                decl = inner.get("ownedTagDecl") or inner.get("decl") or {}
                if inner.get("kind") in ("ElaboratedType", "RecordType") and decl.get("id") in records:
                    self.structs[d["name"]] = records[decl["id"]]
        # cgo built-ins the binding uses (stdlib.h + cgo's own helpers)
        self.funcs.setdefault("malloc", (["C.size_t"], "unsafe.Pointer"))
        self.funcs.setdefault("free", (["unsafe.Pointer"], ""))
        self.funcs["GoString"] = (["*C.char"], "string")


# ----------------------------------------------------------------------------------- Go lexer

KEYWORDS = {"break", "case", "chan", "const", "continue", "default", "defer", "else", "fallthrough", "for",
            "func", "go", "goto", "if", "import", "interface", "map", "package", "range", "return", "select",
            "struct", "switch", "type", "var"}
OPS = sorted(["<<=", ">>=", "&^=", "...", "&&", "||", "<-", "++", "--", "==", "!=", "<=", ">=", ":=", "+=", "-=",
              "*=", "/=", "%=", "&=", "|=", "^=", "<<", ">>", "&^", "+", "-", "*", "/", "%", "&", "|", "^", "<",
              ">", "=", "!", "(", ")", "[", "]", "{", "}", ",", ";", ".", ":", "~"], key=len, reverse=True)


class Tok:
    __slots__ = ("kind", "val", "line")

    def __init__(self, kind, val, line):
        self.kind, self.val, self.line = kind, val, line

    def __repr__(self):
        return "%s:%r@%d" % (self.kind, self.val, self.line)


def lex(src: str) -> list[Tok]:
    toks: list[Tok] = []
    i, n, line = 0, len(src), 1

    def semi_needed():
        if not toks:
            return False
        t = toks[-1]
        return (t.kind in ("ident", "num", "str") and t.val not in KEYWORDS - {"break", "continue", "fallthrough",
                                                                                "return"}) or \
            (t.kind == "op" and t.val in (")", "]", "}", "++", "--"))

    while i < n:
        c = src[i]
        if c == "\n":
            if semi_needed():
                toks.append(Tok("op", ";", line))
            line += 1
            i += 1
        elif c in " \t\r":
            i += 1
        elif src.startswith("//", i):
            j = src.find("\n", i)
            i = n if j < 0 else j
        elif src.startswith("/*", i):
            j = src.find("*/", i + 2)
            j = n if j < 0 else j + 2
            nl = src.count("\n", i, j)
            if nl and semi_needed():
                toks.append(Tok("op", ";", line))
            line += nl
            i = j
        elif c.isalpha() or c == "_":
            j = i
            while j < n and (src[j].isalnum() or src[j] == "_"):
                j += 1
            toks.append(Tok("ident", src[i:j], line))
            i = j
        elif c.isdigit() or (c == "." and i + 1 < n and src[i + 1].isdigit()):
            j = i + 1
            while j < n and (src[j].isalnum() or src[j] in "._" or (src[j] in "+-" and src[j - 1] in "eEpP")):
                j += 1
            toks.append(Tok("num", src[i:j], line))
            i = j
        elif c in "\"'":
            j = i + 1
            while j < n and src[j] != c:
                j += 2 if src[j] == "\\" else 1
            toks.append(Tok("str", src[i:j + 1], line))
            i = j + 1
        elif c == "`":
            j = src.find("`", i + 1)
            line += src.count("\n", i, j)
            toks.append(Tok("str", src[i:j + 1], line))
            i = j + 1
        else:
            for op in OPS:
                if src.startswith(op, i):
                    toks.append(Tok("op", op, line))
                    i += len(op)
                    break
            else:
                raise SyntaxError("line %d: unexpected character %r" % (line, c))
    if semi_needed():
        toks.append(Tok("op", ";", line))
    toks.append(Tok("eof", "", line))
    return toks


# ----------------------------------------------------------------------------------- Go parser
# AST nodes are tuples: (kind, line, ...).  Types are canonical strings ("*arena", "[]C.uint8_t",
# "func(*arena,C.size_t)C.int", "map[*ValSet]*C.tmed_valset"); array lengths that are not a
# literal become "N".

class Parser:
    def __init__(self, toks: list[Tok]):
        self.t, self.p = toks, 0
        self.no_lit = 0  # >0 inside if/for/switch headers: `x {` is not a composite literal

    # -- token helpers
    @property
    def cur(self) -> Tok:
        return self.t[self.p]

    def peek(self, k=1) -> Tok:
        return self.t[min(self.p + k, len(self.t) - 1)]

    def at(self, *vals) -> bool:
        return self.cur.val in vals and self.cur.kind in ("op", "ident")

    def eat(self, val=None) -> Tok:
        t = self.cur
        if val is not None and t.val != val:
            raise SyntaxError("line %d: expected %r, got %r" % (t.line, val, t.val))
        self.p += 1
        return t

    def accept(self, val) -> bool:
        if self.cur.val == val and self.cur.kind in ("op", "ident"):
            self.p += 1
            return True
        return False

    def skip_semis(self):
        while self.at(";"):
            self.p += 1

    # -- file level
    def file(self):
        decls = []
        self.skip_semis()
        if self.accept("package"):
            self.eat()
            self.skip_semis()
        while self.cur.kind != "eof":
            if self.accept("import"):
                if self.accept("("):
                    while not self.accept(")"):
                        self.p += 1
                else:
                    if self.cur.kind == "ident":
                        self.p += 1
                    self.eat()
            elif self.at("func"):
                decls.append(self.funcdecl())
            elif self.at("type", "var", "const"):
                decls.extend(self.gendecl())
            else:
                raise SyntaxError("line %d: unexpected %r at file level" % (self.cur.line, self.cur.val))
            self.skip_semis()
        return decls

    def gendecl(self):
        kw = self.eat().val
        out = []
        if self.accept("("):
            self.skip_semis()
            last_type = None
            while not self.accept(")"):
                d = self.spec(kw, last_type)
                if kw == "const":
                    last_type = d[3] if d[3] else (last_type if not d[4] else None)
                out.append(d)
                self.skip_semis()
        else:
            out.append(self.spec(kw, None))
        return out

    def spec(self, kw, last_type):
        line = self.cur.line
        if kw == "type":
            name = self.eat().val
            self.accept("=")
            if self.at("struct"):
                return ("typedecl", line, name, self.structtype())
            return ("typedecl", line, name, self.type_())
        names = [self.eat().val]
        while self.accept(","):
            names.append(self.eat().val)
        typ = None
        if not self.at("=", ";", ")"):
            typ = self.type_()
        vals = []
        if self.accept("="):
            vals = self.exprlist()
        return ("vardecl", line, names, typ, vals)

    def structtype(self):
        self.eat("struct")
        self.eat("{")
        fields = {}
        self.skip_semis()
        while not self.accept("}"):
            names = [self.eat().val]
            if self.at(";", "}"):   # embedded field
                fields[names[0]] = names[0]
            else:
                while self.accept(","):
                    names.append(self.eat().val)
                t = self.type_()
                for nm in names:
                    fields[nm] = t
            if self.cur.kind == "str":
                self.p += 1
            self.skip_semis()
        return ("struct", fields)

    def funcdecl(self):
        line = self.eat("func").line
        recv = None
        if self.at("("):
            ps = self.params()
            recv = ps[0]
        name = self.eat().val
        params, variadic = self.params(with_variadic=True)
        results = self.results()
        body = self.block() if self.at("{") else None
        return ("func", line, name, recv, params, results, body, variadic)

    def params(self, with_variadic=False):
        """(name|None, type) pairs; Go's `a, b int` grouping resolved."""
        self.eat("(")
        groups = []  # list of token-sliced entries: (maybe_name, type or None)
        variadic = False
        while not self.accept(")"):
            if self.accept("..."):
                variadic = True
            start = self.p
            if self.cur.kind == "ident" and not self.at(*KEYWORDS - {"func", "map", "chan", "struct", "interface"}) \
                    and not (self.peek().val in (",", ")") ) and self.peek().val != ".":
                nm = self.eat().val
                if self.accept("..."):
                    variadic = True
                groups.append((nm, self.type_()))
            else:
                self.p = start
                groups.append((None, self.type_()))
            self.accept(",")
            self.skip_semis()
        # `a, b int`: bare identifiers before a named entry are names of that entry's type
        out, pending = [], []
        named = any(g[0] is not None for g in groups)
        for nm, t in groups:
            if nm is None and named and re.match(r"^\w+$", t):
                pending.append(t)
                continue
            for p in pending:
                out.append((p, t))
            pending = []
            out.append((nm, t))
        for p in pending:
            out.append((None, p))
        return (out, variadic) if with_variadic else out

    def results(self):
        if self.at("("):
            return [t for _, t in self.params()]
        if self.at("{", ";", ")", ",", "]", "}", "=") or self.cur.kind in ("str", "eof"):
            return []
        return [self.type_()]

    # -- types
    def type_(self) -> str:
        t = self.cur
        if self.accept("*"):
            return "*" + self.type_()
        if self.accept("("):
            ty = self.type_()
            self.eat(")")
            return ty
        if self.accept("["):
            if self.accept("]"):
                return "[]" + self.type_()
            if self.accept("..."):
                self.eat("]")
                return "[N]" + self.type_()
            n = self.expr()
            self.eat("]")
            ln = n[2] if n[0] == "num" else "N"
            return "[%s]%s" % (ln, self.type_())
        if self.accept("map"):
            self.eat("[")
            k = self.type_()
            self.eat("]")
            return "map[%s]%s" % (k, self.type_())
        if self.accept("chan"):
            return "chan " + self.type_()
        if self.at("<-"):
            self.eat()
            self.eat("chan")
            return "chan " + self.type_()
        if self.accept("func"):
            ps, _ = self.params(with_variadic=True)
            rs = self.results()
            return functype([p for _, p in ps], rs)
        if self.at("struct"):
            st = self.structtype()
            return "struct{%s}" % ";".join("%s %s" % kv for kv in st[1].items())
        if self.accept("interface"):
            self.eat("{")
            depth = 1
            while depth:
                depth += {"{": 1, "}": -1}.get(self.eat().val, 0)
            return "interface{}"
        if t.kind == "ident":
            self.p += 1
            if self.at(".") and self.peek().kind == "ident":
                self.p += 1
                return t.val + "." + self.eat().val
            return t.val
        raise SyntaxError("line %d: expected a type, got %r" % (t.line, t.val))

    # -- statements
    def block(self):
        self.eat("{")
        saved, self.no_lit = self.no_lit, 0
        stmts = []
        self.skip_semis()
        while not self.accept("}"):
            stmts.append(self.stmt())
            self.skip_semis()
        self.no_lit = saved
        return ("block", stmts)

    def stmt(self):
        t = self.cur
        line = t.line
        if t.kind == "ident":
            v = t.val
            if v in ("var", "const", "type"):
                return ("decl", line, self.gendecl())
            if v == "return":
                self.p += 1
                vals = [] if self.at(";", "}") else self.exprlist()
                return ("return", line, vals)
            if v in ("break", "continue", "goto", "fallthrough"):
                self.p += 1
                if self.cur.kind == "ident":
                    self.p += 1
                return ("branch", line, v)
            if v in ("defer", "go"):
                self.p += 1
                return ("expr", line, self.expr(), v)
            if v == "if":
                return self.ifstmt()
            if v == "for":
                return self.forstmt()
            if v == "switch":
                return self.switchstmt()
            if v == "select":
                return self.selectstmt()
            if self.peek().val == ":" and self.peek().kind == "op" and self.peek(2).val != "=":
                self.p += 2  # label
                return self.stmt() if not self.at("}") else ("empty", line)
        if self.at("{"):
            return self.block()
        return self.simple()

    def simple(self, range_ok=False):
        line = self.cur.line
        if range_ok and self.accept("range"):
            return ("range", line, [], None, self.expr())
        lhs = self.exprlist()
        if self.at(":=", "=", "+=", "-=", "*=", "/=", "%=", "&=", "|=", "^=", "<<=", ">>=", "&^="):
            op = self.eat().val
            if range_ok and self.accept("range"):
                return ("range", line, lhs, op, self.expr())
            rhs = self.exprlist()
            return ("assign", line, lhs, op, rhs)
        if self.at("++", "--"):
            self.eat()
            return ("incdec", line, lhs[0])
        if self.at("<-"):
            self.eat()
            return ("send", line, lhs[0], self.expr())
        return ("expr", line, lhs[0], None)

    def ifstmt(self):
        line = self.eat("if").line
        self.no_lit += 1
        init = None
        s = self.simple()
        if self.accept(";"):
            init, s = s, self.simple()
        self.no_lit -= 1
        cond = s[2]
        body = self.block()
        els = None
        if self.accept("else"):
            els = self.ifstmt() if self.at("if") else self.block()
        return ("if", line, init, cond, body, els)

    def forstmt(self):
        line = self.eat("for").line
        self.no_lit += 1
        init = cond = post = None
        if not self.at("{"):
            s = None if self.at(";") else self.simple(range_ok=True)
            if s is not None and s[0] == "range":
                self.no_lit -= 1
                return ("for", line, s, None, None, self.block())
            if self.accept(";"):
                init = s
                cond = None if self.at(";") else self.simple()
                self.eat(";")
                post = None if self.at("{") else self.simple()
            else:
                cond = s
        self.no_lit -= 1
        return ("for", line, init, cond, post, self.block())

    def switchstmt(self):
        line = self.eat("switch").line
        self.no_lit += 1
        init = tag = None
        if not self.at("{"):
            s = None if self.at(";") else self.simple()
            if self.accept(";"):
                init = s
                s = None if self.at("{") else self.simple()
            tag = s
        self.no_lit -= 1
        self.eat("{")
        cases = []
        self.skip_semis()
        while not self.accept("}"):
            cl = self.cur.line
            if self.accept("default"):
                vals = []
            else:
                self.eat("case")
                vals = self.exprlist()
            self.eat(":")
            body = []
            self.skip_semis()
            while not self.at("case", "default", "}"):
                body.append(self.stmt())
                self.skip_semis()
            cases.append((cl, vals, ("block", body)))
        return ("switch", line, init, tag, cases)

    def selectstmt(self):
        line = self.eat("select").line
        self.eat("{")
        cases = []
        self.skip_semis()
        while not self.accept("}"):
            if self.accept("default"):
                comm = None
            else:
                self.eat("case")
                comm = self.simple()
            self.eat(":")
            body = []
            self.skip_semis()
            while not self.at("case", "default", "}"):
                body.append(self.stmt())
                self.skip_semis()
            cases.append((comm, ("block", body)))
        return ("select", line, cases)

    # -- expressions
    def exprlist(self):
        out = [self.expr()]
        while self.accept(","):
            out.append(self.expr())
        return out

    PREC = {"||": 1, "&&": 2, "==": 3, "!=": 3, "<": 3, "<=": 3, ">": 3, ">=": 3,
            "+": 4, "-": 4, "|": 4, "^": 4, "*": 5, "/": 5, "%": 5, "<<": 5, ">>": 5, "&": 5, "&^": 5}

    def expr(self, prec=1):
        x = self.unary()
        while self.cur.kind == "op" and self.PREC.get(self.cur.val, 0) >= prec:
            op = self.eat()
            y = self.expr(self.PREC[op.val] + 1)
            x = ("binary", op.line, op.val, x, y)
        return x

    def unary(self):
        t = self.cur
        if t.kind == "op" and t.val in ("&", "*", "-", "+", "!", "^", "<-"):
            self.p += 1
            return ("unary", t.line, t.val, self.unary())
        return self.primary()

    def operand(self):
        t = self.cur
        line = t.line
        if t.kind == "num":
            self.p += 1
            return ("num", line, t.val)
        if t.kind == "str":
            self.p += 1
            return ("str", line, t.val)
        if self.at("func"):
            self.p += 1
            ps, _ = self.params(with_variadic=True)
            rs = self.results()
            ft = functype([p for _, p in ps], rs)
            if self.at("{"):
                body = self.block()
                return ("funclit", line, ft, ps, rs, body)
            return ("type", line, ft)
        if self.at("("):
            self.p += 1
            self.no_lit, saved = 0, self.no_lit
            e = self.expr()
            self.no_lit = saved
            self.eat(")")
            return ("paren", line, e)
        if self.at("[", "map", "chan", "struct", "interface"):
            return ("type", line, self.type_())
        if t.kind == "ident":
            self.p += 1
            return ("ident", line, t.val)
        raise SyntaxError("line %d: unexpected %r in expression" % (line, t.val))

    def primary(self):
        x = self.operand()
        while True:
            t = self.cur
            if self.at("."):
                self.p += 1
                if self.accept("("):
                    ty = "type" if self.accept("type") else self.type_()
                    self.eat(")")
                    x = ("assert", t.line, x, ty)
                else:
                    x = ("sel", t.line, x, self.eat().val)
            elif self.at("("):
                self.p += 1
                args = []
                self.no_lit, saved = 0, self.no_lit
                self.skip_semis()
                while not self.accept(")"):
                    if self.at("[", "map", "chan", "func", "*") and _is_type_arg(x):
                        args.append(("type", self.cur.line, self.type_()))
                    else:
                        args.append(self.expr())
                    self.accept("...")
                    self.accept(",")
                    self.skip_semis()
                self.no_lit = saved
                x = ("call", t.line, x, args)
            elif self.at("["):
                self.p += 1
                self.no_lit, saved = 0, self.no_lit
                lo = None if self.at(":") else self.expr()
                if self.accept(":"):
                    hi = None if self.at("]", ":") else self.expr()
                    mx = None
                    if self.accept(":"):
                        mx = self.expr()
                    self.eat("]")
                    x = ("slice", t.line, x, lo, hi, mx)
                else:
                    self.eat("]")
                    x = ("index", t.line, x, lo)
                self.no_lit = saved
            elif self.at("{") and _litable(x) and (self.no_lit == 0 or x[0] == "type"):
                # (in an if/for/switch header only a literal of a TypeName needs parentheses)
                x = ("complit", t.line, type_of_typeexpr(x), self.litbody())
            else:
                return x

    def litbody(self):
        self.eat("{")
        self.no_lit, saved = 0, self.no_lit
        elts = []
        self.skip_semis()
        while not self.accept("}"):
            if self.at("{"):
                v = ("complit", self.cur.line, None, self.litbody())
            else:
                v = self.expr()
            if self.accept(":"):
                k = v
                v = ("complit", self.cur.line, None, self.litbody()) if self.at("{") else self.expr()
                elts.append((k, v))
            else:
                elts.append((None, v))
            self.accept(",")
            self.skip_semis()
        self.no_lit = saved
        return elts


def _is_type_arg(fn):
    return fn[0] == "ident" and fn[2] in ("make", "new")


def _litable(x):
    return x[0] in ("ident", "type") or (x[0] == "sel" and x[2][0] == "ident")


def type_of_typeexpr(x) -> str | None:
    """The canonical type an expression in type position denotes ('C.tmed_x', '*arena', ...)."""
    if x[0] == "ident":
        return x[2]
    if x[0] == "sel" and x[2][0] == "ident":
        return x[2][2] + "." + x[3]
    if x[0] == "type":
        return x[2]
    if x[0] == "unary" and x[2] == "*":
        t = type_of_typeexpr(x[3])
        return "*" + t if t else None
    if x[0] == "paren":
        return type_of_typeexpr(x[2])
    return None


def functype(params, results) -> str:
    r = ",".join(results)
    return "func(%s)%s" % (",".join(params), "(%s)" % r if len(results) > 1 else r)


def split_functype(t: str):
    """'func(A,B)R' -> ([A, B], [R]) (top-level commas only)."""
    assert t.startswith("func(")
    depth, i = 0, 5
    start = 5
    parts = []
    while True:
        c = t[i]
        if c in "([{":
            depth += 1
        elif c in ")]}":
            if depth == 0:
                parts.append(t[start:i])
                break
            depth -= 1
        elif c == "," and depth == 0:
            parts.append(t[start:i])
            start = i + 1
        i += 1
    params = [p for p in parts if p]
    rest = t[i + 1:]
    if rest.startswith("("):
        results = split_functype("func" + rest)[0]
    else:
        results = [rest] if rest else []
    return params, results


# ----------------------------------------------------------------------------------- checker

BUILTIN_TYPES = {"bool", "byte", "int", "int8", "int16", "int32", "int64", "uint", "uint8", "uint16", "uint32",
                 "uint64", "uintptr", "float32", "float64", "string", "error", "rune"}
CONV_TYPES = BUILTIN_TYPES | {"unsafe.Pointer"}


def canon(t):
    if t is None:
        return None
    return t.replace("byte", "uint8") if re.fullmatch(r"[\[\]*N0-9]*byte", t) else t


class Pkg:
    """Declarations of one Go package (the tmedgpu binding)."""

    def __init__(self, decls):
        self.types: dict[str, object] = {}     # name -> ("struct", {field: type}) or underlying type string
        self.methods: dict[str, dict] = {}     # base type -> {name: func decl}
        self.funcs: dict[str, tuple] = {}
        self.vars: dict[str, str | None] = {}
        for d in decls:
            if d[0] == "typedecl":
                self.types[d[2]] = d[3]
            elif d[0] == "vardecl":
                for nm in d[2]:
                    self.vars[nm] = d[3]
            elif d[0] == "func":
                if d[3] is not None:
                    base = d[3][1].lstrip("*")
                    self.methods.setdefault(base, {})[d[2]] = d
                else:
                    self.funcs[d[2]] = d

    def struct_fields(self, t):
        t = t.lstrip("*") if t else t
        st = self.types.get(t)
        return st[1] if isinstance(st, tuple) and st[0] == "struct" else None


class Checker:
    def __init__(self, header: Header, pkg: Pkg, where: str, pkgname: str | None = None, ext: Pkg | None = None):
        """pkgname None: the code is package tmedgpu itself (pkg); else code of another package that
        imports tmedgpu as `pkgname` (ext = the tmedgpu declarations)."""
        self.h, self.pkg, self.where = header, pkg, where
        self.ext_name, self.ext = pkgname, ext
        self.errors: list[str] = []
        self.declared: list = []   # (scope, name, line) of local variables
        self.stats = dict.fromkeys(("c_calls", "c_args", "c_args_typed", "go_calls", "go_args", "go_args_typed"), 0)
        self.used: set = set()

    def err(self, line, msg):
        self.errors.append("%s:%d: %s" % (self.where, line, msg))

    # -- type helpers
    def qual(self, t):
        """A tmedgpu type named from outside the package: 'tmedgpu.ValSet' -> 'ValSet' (its own pkg)."""
        if t and self.ext_name:
            return re.sub(r"\b%s\." % re.escape(self.ext_name), "", t)
        return t

    def own(self):
        return self.ext if self.ext_name else self.pkg

    def fields_of(self, t):
        """(fields dict, is_c) of struct type t (pointer stripped), or (None, False)."""
        if t is None:
            return None, False
        b = t.lstrip("*")
        if b.startswith("C.") and b[2:] in self.h.structs:
            return self.h.structs[b[2:]], True
        f = self.own().struct_fields(self.qual(b))
        return f, False

    def elem(self, t):
        if t is None:
            return None
        t = t.lstrip("*") if t.startswith("*[") else t
        m = re.match(r"^\[(\w*)\](.*)$", t)
        if m:
            return m.group(2)
        m = re.match(r"^map\[.*?\](.*)$", t)
        if m:
            return m.group(1)
        if t.startswith("chan "):
            return t[5:]
        if t == "string":
            return "uint8"
        return None

    def compatible(self, want, got):
        if want is None or got is None or want == "" or got == "":
            return True
        want, got = canon(self.qual(want)), canon(self.qual(got))
        if want == got or got == "untyped" or want in ("interface{}", "error"):
            return True
        if got == "nil":
            return want.startswith(("*", "[]", "map[", "chan ", "func(")) or want in ("unsafe.Pointer", "error")
        return False

    # -- walking
    def check_func(self, fdecl, outer=None):
        _, line, name, recv, params, results, body, variadic = fdecl
        scope = dict(outer or {})
        if recv and recv[0]:
            scope[recv[0]] = recv[1]
        for nm, t in params:
            if nm:
                scope[nm] = t
        if body:
            self.block(body, [scope], results)
        self.report_unused()

    def lookup(self, scopes, name, mark=True):
        for s in reversed(scopes):
            if name in s:
                if mark:
                    self.used.add((id(s), name))
                return s[name]
        return self.pkg.vars.get(name) if not self.ext_name else None

    def block(self, blk, scopes, results, nilvars=None):
        scopes = scopes + [{}]
        nil = dict(nilvars or {})   # var -> err var it came with (may be nil while err may be non-nil)
        for st in blk[1]:
            self.stmt(st, scopes, results, nil)
        return nil

    def declare(self, scopes, name, t, line=0):
        if name != "_":
            scopes[-1][name] = t
            self.declared.append((scopes[-1], name, line))

    def report_unused(self):
        """Go rejects a local variable that is declared and never used (a compile error)."""
        for sc, name, line in self.declared:
            if (id(sc), name) not in self.used and line:
                self.err(line, "%s declared and not used" % name)
        self.declared = []

    def stmt(self, st, scopes, results, nil):
        k = st[0]
        if k == "expr":
            self.expr(st[2], scopes, nil)
        elif k == "assign":
            _, line, lhs, op, rhs = st
            rts = [self.expr(r, scopes, nil) for r in rhs]
            if len(rhs) == 1 and len(lhs) > 1:
                rts = self.multi(rhs[0], scopes, len(lhs))
            for i, l in enumerate(lhs):
                rt = rts[i] if i < len(rts) else None
                if op == ":=" and l[0] == "ident":
                    if rt == "untyped":  # an untyped constant's default type
                        r = rhs[i] if len(rhs) == len(lhs) else None
                        rt = "int" if r is not None and r[0] == "num" and re.fullmatch(r"[0-9xXa-fA-F_]+", r[2]) \
                            else ("string" if r is not None and r[0] == "str" else None)
                    if l[2] not in scopes[-1]:
                        self.declare(scopes, l[2], rt, line)
                elif op == "=" and l[0] == "ident":
                    lt = self.lookup(scopes, l[2], mark=False)
                    if lt is None and l[2] != "_" and not self.ext_name and l[2] in self.pkg.vars:
                        lt = self.pkg.vars[l[2]]
                    if not self.compatible(lt, rt):
                        self.err(line, "assigning %s to %s of type %s" % (rt, self.show(l), lt))
                else:
                    lt = self.expr(l, scopes, nil, lvalue=True)
                    if op == "=" and not self.compatible(lt, rt):
                        self.err(line, "assigning %s to %s of type %s" % (rt, self.show(l), lt))
                # nil tracking: `p, err := f()` with f returning (*T, error)
                if l[0] == "ident":
                    nil.pop(l[2], None)
            if len(lhs) == 2 and len(rhs) == 1 and lhs[0][0] == "ident" and lhs[1][0] == "ident" \
                    and rhs[0][0] == "call":
                rs = self.results_of(rhs[0], scopes)
                if rs and len(rs) == 2 and rs[1] == "error" and rs[0].startswith("*"):
                    nil[lhs[0][2]] = lhs[1][2]
            if len(lhs) == len(rhs):
                for l, r in zip(lhs, rhs):
                    if l[0] == "ident" and r[0] == "ident" and r[2] in nil:
                        nil[l[2]] = nil[r[2]]
        elif k == "incdec":
            self.expr(st[2], scopes, nil)
        elif k == "send":
            self.expr(st[2], scopes, nil)
            self.expr(st[3], scopes, nil)
        elif k == "decl":
            for d in st[2]:
                if d[0] == "vardecl":
                    vts = [self.expr(v, scopes, nil) for v in d[4]]
                    for i, nm in enumerate(d[2]):
                        self.declare(scopes, nm, d[3] or (vts[i] if i < len(vts) else None), d[1])
        elif k == "return":
            vals = st[2]
            ts = [self.expr(v, scopes, nil) for v in vals]
            if results is not None and vals and not (len(vals) == 1 and len(results) > 1):
                if len(vals) != len(results):
                    self.err(st[1], "returns %d values, the function declares %d" % (len(vals), len(results)))
                else:
                    for want, got, v in zip(results, ts, vals):
                        if not self.compatible(want, got):
                            self.err(st[1], "returns %s as %s (want %s)" % (self.show(v), got, want))
        elif k == "block":
            self.block(st, scopes, results, nil)
        elif k == "if":
            self.ifstmt(st, scopes, results, nil)
        elif k == "for":
            _, line, init, cond, post, body = st
            sc = scopes + [{}]
            if init is not None and init[0] == "range":
                _, rl, lhs, op, x = init
                xt = self.expr(x, sc, nil)
                kt, vt = ("int" if xt else None), self.elem(xt)
                if xt and xt.startswith("map["):
                    kt = xt[4:].split("]")[0]
                if xt and xt.startswith("chan "):
                    kt = vt
                for i, l in enumerate(lhs):
                    if l[0] == "ident" and op == ":=":
                        self.declare(sc, l[2], kt if i == 0 else vt, rl)
                    elif l[0] == "ident":
                        self.lookup(sc, l[2], mark=False)
            else:
                for s in (init, cond, post):
                    if s is not None:
                        self.stmt(s, sc, results, nil)
            self.block(body, sc, results, nil)
        elif k == "switch":
            _, line, init, tag, cases = st
            sc = scopes + [{}]
            if init is not None:
                self.stmt(init, sc, results, nil)
            if tag is not None:
                self.stmt(tag, sc, results, nil)
            for _, vals, body in cases:
                for v in vals:
                    self.expr(v, sc, nil)
                self.block(body, sc, results, nil)
        elif k == "select":
            for comm, body in st[2]:
                sc = scopes + [{}]
                if comm is not None:
                    self.stmt(comm, sc, results, nil)
                self.block(body, sc, results, nil)

    def ifstmt(self, st, scopes, results, nil):
        _, line, init, cond, body, els = st
        sc = scopes + [{}]
        if init is not None:
            self.stmt(init, sc, results, nil)
        self.expr(cond, sc, nil)
        errvar, op = None, None
        if cond[0] == "binary" and cond[2] in ("==", "!=") and cond[3][0] == "ident" and cond[4] == ("ident", cond[4][1], "nil"):
            errvar, op = cond[3][2], cond[2]
        inner = dict(nil)
        if op == "==":  # err == nil: the values that came with it are usable inside
            inner = {v: e for v, e in nil.items() if e != errvar}
        self.block(body, sc, results, inner)
        if els is not None:
            other = dict(nil)
            if op == "!=":
                other = {v: e for v, e in nil.items() if e != errvar}
            if els[0] == "if":
                self.ifstmt(els, sc, results, other)
            else:
                self.block(els, sc, results, other)
        if op == "!=" and terminates(body):
            for v in [v for v, e in nil.items() if e == errvar]:
                del nil[v]

    def multi(self, x, scopes, n):
        """Types of a multi-value right-hand side."""
        if x[0] == "call":
            rs = self.results_of(x, scopes)
            if rs:
                return rs
        if x[0] == "index":
            return [self.expr(x, scopes, {}), "bool"]
        if x[0] == "unary" and x[2] == "<-":
            return [self.expr(x, scopes, {}), "bool"]
        if x[0] == "assert":
            return [self.expr(x, scopes, {}), "bool"]
        return [None] * n

    def results_of(self, call, scopes):
        fn = call[2]
        sig = self.signature(fn, scopes)
        return sig[1] if sig else None

    def signature(self, fn, scopes):
        """(params, results, variadic, kind, name) of the callee, or None."""
        own = self.own()
        if fn[0] == "ident":
            t = self.lookup(scopes, fn[2])
            if t and t.startswith("func("):
                ps, rs = split_functype(t)
                return ps, rs, False, "var", fn[2]
            if not self.ext_name and fn[2] in own.funcs:
                d = own.funcs[fn[2]]
                return [p for _, p in d[4]], d[5], d[7], "func", fn[2]
            return None
        if fn[0] == "sel":
            base = fn[2]
            if base[0] == "ident" and base[2] == "C" and self.lookup(scopes, "C") is None:
                return None
            if self.ext_name and base[0] == "ident" and base[2] == self.ext_name and self.lookup(scopes, base[2]) is None:
                d = own.funcs.get(fn[3])
                if d is None:
                    return None
                return [p for _, p in d[4]], [self.extq(r) for r in d[5]], d[7], "func", fn[3]
            bt = self.expr(base, scopes, {})
            if bt:
                b = self.qual(bt).lstrip("*")
                d = own.methods.get(b, {}).get(fn[3])
                if d is not None:
                    rs = [self.extq(r) for r in d[5]] if self.ext_name else d[5]
                    ps = [self.extq(p) for _, p in d[4]] if self.ext_name else [p for _, p in d[4]]
                    return ps, rs, d[7], "method", b + "." + fn[3]
        return None

    def extq(self, t):
        """A type of the tmedgpu package seen from the importing package."""
        if not t or not self.ext_name:
            return t
        m = re.match(r"^([\[\]*N0-9]*)(\w+)$", t)
        if m and m.group(2) in self.own().types:
            return m.group(1) + self.ext_name + "." + m.group(2)
        return t

    def show(self, x):
        if x[0] == "ident":
            return x[2]
        if x[0] == "sel":
            return self.show(x[2]) + "." + x[3]
        if x[0] == "unary":
            return x[2] + self.show(x[3])
        if x[0] == "index":
            return self.show(x[2]) + "[...]"
        if x[0] == "call":
            return self.show(x[2]) + "(...)"
        return x[0]

    def expr(self, x, scopes, nil, lvalue=False):
        k = x[0]
        if k == "num":
            return "untyped"
        if k == "str":
            return "untyped"
        if k == "ident":
            if x[2] == "nil":
                return "nil"
            if x[2] in ("true", "false"):
                return "bool"
            t = self.lookup(scopes, x[2])
            if t is None and not self.ext_name and x[2] in self.pkg.funcs:
                d = self.pkg.funcs[x[2]]
                return functype([p for _, p in d[4]], d[5])
            return t
        if k == "paren":
            return self.expr(x[2], scopes, nil)
        if k == "type":
            return None
        if k == "funclit":
            _, line, ft, ps, rs, body = x
            sc = scopes + [{nm: t for nm, t in ps if nm}]
            self.block(body, sc, rs, {})
            return ft
        if k == "unary":
            t = self.expr(x[3], scopes, nil)
            if x[2] == "&":
                if x[3][0] == "complit":
                    return "*" + t if t else None
                return "*" + t if t else None
            if x[2] == "*":
                return t[1:] if t and t.startswith("*") else None
            if x[2] == "<-":
                return self.elem(t)
            if x[2] == "!":
                return "bool"
            return t
        if k == "binary":
            a = self.expr(x[3], scopes, nil)
            b = self.expr(x[4], scopes, nil)
            if x[2] in ("==", "!=", "<", "<=", ">", ">=", "&&", "||"):
                return "bool"
            if x[2] in ("<<", ">>"):
                return a
            return a if a not in (None, "untyped") else b
        if k == "index":
            t = self.expr(x[2], scopes, nil)
            self.expr(x[3], scopes, nil)
            return self.elem(t)
        if k == "slice":
            t = self.expr(x[2], scopes, nil)
            for e in x[3:]:
                if e is not None:
                    self.expr(e, scopes, nil)
            if t is None:
                return None
            if t == "string":
                return t
            e = self.elem(t)
            return "[]" + e if e else None
        if k == "assert":
            self.expr(x[2], scopes, nil)
            return x[3] if x[3] != "type" else None
        if k == "complit":
            return self.complit(x, scopes, nil)
        if k == "sel":
            return self.selector(x, scopes, nil, lvalue)
        if k == "call":
            return self.call(x, scopes, nil)
        return None

    def complit(self, x, scopes, nil, t=None):
        _, line, lt, elts = x
        lt = lt or t
        fields, is_c = self.fields_of(lt) if lt and not lt.startswith(("[", "map[", "*[")) else (None, False)
        if lt and self.ext_name and lt.startswith(self.ext_name + ".") and fields is None:
            if lt[len(self.ext_name) + 1:] not in self.own().types:
                self.err(line, "%s is not a type of package %s" % (lt, self.ext_name))
        for key, v in elts:
            want = None
            if key is not None and key[0] == "ident" and fields is not None:
                if key[2] not in fields:
                    self.err(line, "%s has no field %s" % (lt, key[2]))
                else:
                    want = fields[key[2]]
                    if self.ext_name and not key[2][0].isupper() and not is_c:
                        self.err(line, "field %s of %s is unexported" % (key[2], lt))
            elif key is not None:
                self.expr(key, scopes, nil)
            if v[0] == "complit" and v[2] is None:
                et = want or (self.elem(lt) if lt else None)
                vt = self.complit(v, scopes, nil, et)
            else:
                vt = self.expr(v, scopes, nil)
            if key is not None and fields is not None and key[2] in fields:
                if not self.compatible(self.extq(want) if self.ext_name and not is_c else want, vt):
                    self.err(line, "%s{%s: ...} given %s (field type %s)" % (lt, key[2], vt, want))
        return lt

    def selector(self, x, scopes, nil, lvalue):
        _, line, base, name = x
        if base[0] == "ident" and base[2] == "C" and self.lookup(scopes, "C") is None:
            if name.startswith("TMED_") or name.isupper():
                if name not in self.h.macros:
                    self.err(line, "C.%s is not defined in include/tmed25519.h" % name)
                return "untyped"
            return None
        if base[0] == "ident" and base[2] == "unsafe":
            return None
        if self.ext_name and base[0] == "ident" and base[2] == self.ext_name and self.lookup(scopes, base[2]) is None:
            own = self.own()
            if not name[0].isupper():
                self.err(line, "%s.%s is unexported" % (self.ext_name, name))
            elif name not in own.funcs and name not in own.types and name not in own.vars \
                    and not self.ext_const(name):
                self.err(line, "%s.%s is not declared in tmedgpu.go" % (self.ext_name, name))
            if name in own.vars:
                return self.extq(own.vars[name])
            if name in own.funcs:
                d = own.funcs[name]
                return functype([self.extq(p) for _, p in d[4]], [self.extq(r) for r in d[5]])
            return self.ext_const(name)
        if base[0] == "ident" and base[2] in nil and (self.lookup(scopes, base[2]) or "").startswith(("*", self.ext_name or "\0")):
            self.err(line, "%s may be nil here: it came with %s, which is not checked on this path"
                     % (base[2], nil[base[2]]))
        bt = self.expr(base, scopes, nil)
        if bt is None:
            return None
        fields, is_c = self.fields_of(bt)
        own = self.own()
        b = self.qual(bt).lstrip("*")
        if own.methods.get(b, {}).get(name) is not None:
            d = own.methods[b][name]
            if self.ext_name and not name[0].isupper():
                self.err(line, "method %s.%s is unexported" % (b, name))
            return functype([p for _, p in d[4]], d[5])
        if fields is not None:
            if name not in fields:
                self.err(line, "%s has no field or method %s" % (bt, name))
                return None
            if self.ext_name and not is_c and not name[0].isupper():
                self.err(line, "field %s of %s is unexported" % (name, bt))
            ft = fields[name]
            return self.extq(ft) if self.ext_name and not is_c else ft
        if b in own.types or (bt.startswith("C.") and bt[2:] not in self.h.structs and bt.startswith("C.tmed_")):
            if b in own.types and not isinstance(own.types[b], tuple):
                return None  # a named non-struct type (Mode): no fields
            self.err(line, "%s has no field or method %s" % (bt, name))
        return None

    def ext_const(self, name):
        """Type of an exported tmedgpu constant (declared in a const block), else None."""
        return self.own().vars.get(name, None) or ("untyped" if name in self.own().vars else None)

    def call(self, x, scopes, nil):
        _, line, fn, args = x
        # conversions: T(x), (*T)(p), []byte(s)
        tt = None
        if fn[0] == "type":
            tt = fn[2]
        elif fn[0] == "paren":
            tt = type_of_typeexpr(fn[2])
        elif fn[0] == "ident" and fn[2] in CONV_TYPES and self.lookup(scopes, fn[2]) is None:
            tt = fn[2]
        elif fn[0] == "ident" and fn[2] in self.own().types and self.lookup(scopes, fn[2]) is None and not self.ext_name:
            tt = fn[2]
        elif fn[0] == "sel" and fn[2][0] == "ident" and fn[2][2] == "C" and not (fn[3] in self.h.funcs):
            tt = "C." + fn[3]
            if fn[3] not in ("int", "uint", "char", "size_t", "uint8_t", "uint32_t", "int32_t", "int64_t",
                             "uint64_t", "float", "double") and fn[3] not in self.h.structs:
                self.err(line, "C.%s is not declared in include/tmed25519.h (neither a function nor a type)" % fn[3])
                tt = "?"
        elif fn[0] == "sel" and fn[2][0] == "ident" and fn[2][2] == "unsafe" and fn[3] == "Pointer":
            tt = "unsafe.Pointer"
        if tt is not None:
            for a in args:
                self.expr(a, scopes, nil)
            return tt if tt != "?" else None
        if fn[0] == "ident" and self.lookup(scopes, fn[2]) is None:
            b = fn[2]
            ats = [self.expr(a, scopes, nil) if a[0] != "type" else a[2] for a in args]
            if b == "len" or b == "cap" or b == "copy":
                return "int"
            if b == "make":
                return ats[0] if ats else None
            if b == "new":
                return "*" + ats[0] if ats and ats[0] else None
            if b == "append":
                return ats[0] if ats else None
            if b in ("panic", "delete", "close", "print", "println"):
                return None
        if fn[0] == "sel" and fn[2][0] == "ident" and fn[2][2] == "unsafe":
            ats = [self.expr(a, scopes, nil) for a in args]
            if fn[3] == "Slice":
                return "[]" + ats[0][1:] if ats and ats[0] and ats[0].startswith("*") else None
            if fn[3] == "Add":
                return "unsafe.Pointer"
            if fn[3] in ("Sizeof", "Offsetof", "Alignof"):
                return "uintptr"
            return None
        if fn[0] == "sel" and fn[2][0] == "ident" and fn[2][2] == "C" and self.lookup(scopes, "C") is None:
            return self.c_call(x, scopes, nil)
        sig = self.signature(fn, scopes)
        if fn[0] == "sel":
            self.selector(fn, scopes, nil, False)
        else:
            self.expr(fn, scopes, nil)
        ats = [self.expr(a, scopes, nil) for a in args]
        if sig is None:
            return None
        ps, rs, variadic, kind, name = sig
        self.stats["go_calls"] += 1
        self.stats["go_args"] += len(args)
        self.stats["go_args_typed"] += sum(1 for t in ats if t not in (None, "untyped"))
        spread = any(a[0] == "call" and (self.results_of(a, scopes) or [None, None]).__len__() > 1 for a in args) \
            and len(args) == 1
        if not spread:
            if (len(args) != len(ps) and not variadic) or (variadic and len(args) < len(ps) - 1):
                self.err(line, "%s %s takes %d arguments, called with %d" % (kind, name, len(ps), len(args)))
            else:
                for i, (a, at) in enumerate(zip(args, ats)):
                    want = ps[i] if i < len(ps) else None
                    if variadic and i >= len(ps) - 1:
                        want = None
                    if not self.compatible(want, at):
                        self.err(line, "argument %d of %s %s: %s is %s, the parameter is %s"
                                 % (i + 1, kind, name, self.show(a), at, want))
        return rs[0] if len(rs) == 1 else (None if not rs else None)

    def c_call(self, x, scopes, nil):
        _, line, fn, args = x
        name = fn[3]
        ats = [self.expr(a, scopes, nil) for a in args]
        if name not in self.h.funcs:
            self.err(line, "C.%s is not declared in include/tmed25519.h" % name)
            return None
        ps, res = self.h.funcs[name]
        self.stats["c_calls"] += 1
        self.stats["c_args"] += len(args)
        self.stats["c_args_typed"] += sum(1 for t in ats if t not in (None, "untyped"))
        if len(args) != len(ps):
            self.err(line, "C.%s takes %d arguments (include/tmed25519.h), called with %d" % (name, len(ps), len(args)))
        else:
            for i, (a, at) in enumerate(zip(args, ats)):
                if not self.compatible(ps[i], at):
                    self.err(line, "argument %d of C.%s: %s is %s, the header's parameter is %s"
                             % (i + 1, name, self.show(a), at, ps[i]))
        return res or None


def terminates(blk) -> bool:
    if not blk[1]:
        return False
    last = blk[1][-1]
    if last[0] in ("return",):
        return True
    if last[0] == "branch" and last[2] in ("break", "continue", "goto"):
        return True
    if last[0] == "expr" and last[2][0] == "call" and last[2][2][0] == "ident" and last[2][2][2] == "panic":
        return True
    return False


# ----------------------------------------------------------------------------------- drivers

def parse_go(src: str):
    return Parser(lex(src)).file()


def check_preamble(go_src: str, go_dir: str, where="tmedgpu.go"):
    """The cgo preamble's -I / -L directories (relative to ${SRCDIR}) exist and hold the header it
    includes and the library it links."""
    errs = []
    m = re.search(r"/\*(.*?)\*/\s*import \"C\"", go_src, re.S)
    if not m:
        return ["%s: no cgo preamble before import \"C\"" % where]
    pre = m.group(1)
    incs = re.findall(r"#include \"([^\"]+)\"", pre)
    for flag, kind in (("-I", "include"), ("-L", "lib")):
        for d in re.findall(r"%s\$\{SRCDIR\}(\S+)" % flag, pre):
            path = os.path.normpath(go_dir + d)
            if not os.path.isdir(path):
                errs.append("%s: cgo %s directory %s does not exist" % (where, flag, path))
            elif kind == "include":
                for h in incs:
                    if not os.path.exists(os.path.join(path, h)):
                        errs.append("%s: %s not found in the cgo include directory %s" % (where, h, path))
    for lib in re.findall(r"-l(\w+)", pre):
        dirs = [os.path.normpath(go_dir + d) for d in re.findall(r"-L\$\{SRCDIR\}(\S+)", pre)]
        srcs = [os.path.join(d, "lib%s.so" % lib) for d in dirs]
        # the library is a build product (make -C tendermint-fork_amd); its Makefile target must exist
        if not any(os.path.exists(x) for x in srcs) and not any(
                os.path.exists(os.path.join(os.path.dirname(d), "Makefile")) for d in dirs):
            errs.append("%s: -l%s: neither built nor buildable from the -L directories" % (where, lib))
    return errs


def check_binding(go_src: str, header: Header, where="tmedgpu.go", extra=()):
    """The package's main file plus `extra` [(name, source)] files of the same package (its
    _test.go): one declaration set, every function checked, errors named by file."""
    files = [(where, parse_go(go_src))] + [(w, parse_go(src)) for w, src in extra]
    pkg = Pkg([d for _, ds in files for d in ds])
    errors = []
    for w, decls in files:
        ck = Checker(header, pkg, w)
        for d in decls:
            if d[0] == "func":
                ck.check_func(d)
            elif d[0] == "vardecl":
                for v in d[4]:
                    ck.expr(v, [{}], {})
        if w == where:
            check_binding.stats = ck.stats
        errors += ck.errors
    return errors, pkg


def go_blocks(md: str):
    """(first line number, text) of every ```go block of a markdown file."""
    out = []
    lines = md.split("\n")
    i = 0
    while i < len(lines):
        if lines[i].strip() == "```go":
            j = i + 1
            while lines[j].strip() != "```":
                j += 1
            out.append((i + 2, "\n".join(lines[i + 1:j])))
            i = j
        i += 1
    return out


# names the INTEGRATION.md fragments use without declaring them
SNIPPET_SCOPE = {"eng": "*tmedgpu.Engine"}


def check_snippets(md: str, header: Header, pkg: Pkg, where="INTEGRATION.md"):
    """The Go snippets of INTEGRATION.md as code of package types importing tmedgpu."""
    errors = []
    for first, text in go_blocks(md):
        ck = Checker(header, Pkg([]), "%s(block at line %d)" % (where, first - 1), pkgname="tmedgpu", ext=pkg)
        try:
            decls = Parser(lex(text)).file()
            body = None
        except SyntaxError:
            decls = None
        if decls is None:  # a statement fragment: check it as the body of a function
            p = Parser(lex("{\n" + text + "\n}"))
            try:
                body = p.block()
            except SyntaxError as e:
                errors.append("%s: does not parse as Go: %s" % (ck.where, e))
                continue
            ck.block(body, [dict(SNIPPET_SCOPE)], None)
            ck.declared = []  # a fragment's variables are used by the elided code around it
        else:
            for d in decls:
                if d[0] == "func":
                    ck.check_func(d)
        # line numbers inside a block are relative to it: shift them to the file's
        for e in ck.errors:
            m = re.match(r"^(.*?\)):(\d+): (.*)$", e)
            if m:
                ln = int(m.group(2)) + first - 1 - (1 if decls is None else 0)
                errors.append("%s:%d: %s" % (where, ln, m.group(3)))
            else:
                errors.append(e)
    return errors


def run(go_src=None, md_src=None, header_text=None):
    header = Header(text=header_text) if header_text is not None else Header()
    if go_src is None:
        with open(GO_FILE) as f:
            go_src = f.read()
    if md_src is None:
        with open(INTEGRATION) as f:
            md_src = f.read()
    errs = check_preamble(go_src, os.path.dirname(GO_FILE))
    extra = []
    test_file = GO_FILE[:-3] + "_test.go"
    if os.path.exists(test_file):
        with open(test_file) as f:
            extra.append((os.path.basename(test_file), f.read()))
    e2, pkg = check_binding(go_src, header, extra=extra)
    errs += e2 + check_snippets(md_src, header, pkg)
    return errs


def main():
    errs = run()
    for e in errs:
        print(e)
    print("go_cgo_check: %d finding(s); binding coverage %s" % (len(errs), check_binding.stats), file=sys.stderr)
    return 1 if errs else 0


if __name__ == "__main__":
    sys.exit(main())
