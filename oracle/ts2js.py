#!/usr/bin/env python3
"""TEST INFRASTRUCTURE ONLY -- TypeScript-subset -> ES-module JavaScript stripper.

The reference merge-tree (packages/dds/merge-tree/src/*.ts, TypeScript ~3.7) cannot be
built here: there is no `tsc`, no node_modules and no network.  Node v12 *is* present, so
this script removes the TypeScript-only syntax from the reference's own source files and
writes runnable `.mjs` files into `oracle/_ref/` (git-ignored, never shipped to the GPU
box).  The result is the *reference itself* executing, used only to generate and pin the
golden vectors under tests/golden/.  Nothing in the product imports this.

What is handled (the subset the merge-tree package uses):
  * type annotations on parameters, variables, class fields, return types
  * interfaces, type aliases, `declare`, `implements`, access modifiers, `abstract`
  * generics on declarations, calls and `new`, `<T>x` and `x as T` assertions, `x!`
  * parameter properties and initialised instance fields (moved into the constructor
    after `super()`, parameter properties first -- TS 3.7 `useDefineForClassFields=false`)
  * uninitialised field declarations are elided (TS 3.7 emits nothing for them)
  * enums / const enums -> runtime objects
  * `?.` and `??` down-levelled (Node 12 has neither)
  * imports: type-only specifiers and specifiers unused in value positions are elided,
    matching tsc's import elision (this matters for module-cycle evaluation order).
"""
import os
import re
import sys
import json

# '>' is always lexed alone (or as '>=') so that nested generics `A<B<C>>` close
# correctly; shift operators are re-assembled from adjacent tokens in the parser.
PUNCT = [
    "...", "===", "!==", "**=", "<<=",
    "=>", "==", "!=", "<=", ">=", "&&", "||", "??", "?.", "++", "--", "+=", "-=", "*=", "/=",
    "%=", "&=", "|=", "^=", "<<", "**",
    "{", "}", "(", ")", "[", "]", ";", ",", "<", ">", "+", "-", "*", "/", "%", "&", "|",
    "^", "!", "~", "?", ":", "=", ".", "@", "#",
]
KEYWORDS_BEFORE_REGEX = {"return", "typeof", "case", "do", "else", "in", "of", "new",
                         "delete", "void", "throw", "instanceof", "yield", "await"}


class Tok:
    __slots__ = ("k", "v", "s", "e", "nl")

    def __init__(self, k, v, s, e, nl):
        self.k, self.v, self.s, self.e, self.nl = k, v, s, e, nl

    def __repr__(self):
        return f"{self.k}:{self.v!r}@{self.s}"


def lex(src):
    toks = []
    i, n = 0, len(src)
    nl = False
    while i < n:
        c = src[i]
        if c in " \t\r\n﻿":
            if c == "\n":
                nl = True
            i += 1
            continue
        if src.startswith("//", i):
            j = src.find("\n", i)
            i = n if j < 0 else j
            continue
        if src.startswith("/*", i):
            j = src.find("*/", i + 2)
            if "\n" in src[i:j]:
                nl = True
            i = j + 2
            continue
        s = i
        if c.isalpha() or c in "_$":
            while i < n and (src[i].isalnum() or src[i] in "_$"):
                i += 1
            toks.append(Tok("id", src[s:i], s, i, nl))
        elif c.isdigit() or (c == "." and i + 1 < n and src[i + 1].isdigit()):
            m = re.compile(r"0[xX][0-9a-fA-F_]+n?|0[bB][01_]+n?|0[oO][0-7_]+n?|"
                           r"(\d[\d_]*)?(\.\d[\d_]*)?([eE][+-]?\d+)?n?").match(src, i)
            i = m.end() if m.end() > i else i + 1
            toks.append(Tok("num", src[s:i], s, i, nl))
        elif c in "'\"":
            i += 1
            while src[i] != c:
                i += 2 if src[i] == "\\" else 1
            i += 1
            toks.append(Tok("str", src[s:i], s, i, nl))
        elif c == "`":
            i = skip_template(src, i)
            toks.append(Tok("tmpl", src[s:i], s, i, nl))
        elif c == "/" and regex_allowed(toks):
            i += 1
            in_class = False
            while True:
                ch = src[i]
                if ch == "\\":
                    i += 2
                    continue
                if ch == "[":
                    in_class = True
                elif ch == "]":
                    in_class = False
                elif ch == "/" and not in_class:
                    break
                i += 1
            i += 1
            while i < n and src[i].isalpha():
                i += 1
            toks.append(Tok("re", src[s:i], s, i, nl))
        else:
            for p in PUNCT:
                if src.startswith(p, i):
                    if p == "?." and i + 2 < n and src[i + 2].isdigit():
                        continue
                    i += len(p)
                    toks.append(Tok("p", p, s, i, nl))
                    break
            else:
                raise SyntaxError(f"bad char {c!r} at {i}")
        nl = False
    toks.append(Tok("eof", "", n, n, True))
    return toks


def skip_template(src, i):
    i += 1
    while src[i] != "`":
        if src[i] == "\\":
            i += 2
            continue
        if src.startswith("${", i):
            i += 2
            depth = 1
            while depth:
                ch = src[i]
                if ch in "'\"":
                    q = ch
                    i += 1
                    while src[i] != q:
                        i += 2 if src[i] == "\\" else 1
                    i += 1
                    continue
                if ch == "`":
                    i = skip_template(src, i)
                    continue
                if ch == "{":
                    depth += 1
                elif ch == "}":
                    depth -= 1
                i += 1
            continue
        i += 1
    return i + 1


def regex_allowed(toks):
    if not toks:
        return True
    t = toks[-1]
    if t.k in ("num", "str", "tmpl", "re"):
        return False
    if t.k == "id":
        return t.v in KEYWORDS_BEFORE_REGEX
    return t.v not in (")", "]", "}")


ASSIGN_OPS = {"=", "+=", "-=", "*=", "/=", "%=", "&=", "|=", "^=", "<<=", ">>=", ">>>=", "**="}
BIN_PREC = {
    "??": 1, "||": 1, "&&": 2, "|": 3, "^": 4, "&": 5,
    "==": 6, "!=": 6, "===": 6, "!==": 6,
    "<": 7, ">": 7, "<=": 7, ">=": 7, "instanceof": 7, "in": 7, "as": 7,
    "<<": 8, ">>": 8, ">>>": 8, "+": 9, "-": 9, "*": 10, "/": 10, "%": 10, "**": 11,
}
MODIFIERS = {"public", "private", "protected", "readonly", "static", "abstract", "declare",
             "async", "override"}


class Transpiler:
    def __init__(self, src, name=""):
        self.src = src
        self.name = name
        self.t = lex(src)
        self.i = 0
        self.edits = []          # list of [start, end, text]
        self.imports = []        # (kind, local, imported, module)
        self.exported = set()    # value names exported by declarations / lists
        self.reexports = []      # ("*", module) or ("names", [(local, exported)], module)

    # ------------------------------------------------------------------ edits
    def edit(self, s, e, text=""):
        self.edits.append([s, e, text])

    def render(self, s, e):
        out, pos = [], s
        for es, ee, tx in sorted((x for x in self.edits if x[0] >= s and x[1] <= e),
                                 key=lambda x: (x[0], x[1])):
            if es < pos:
                continue
            out.append(self.src[pos:es])
            out.append(tx)
            pos = ee
        out.append(self.src[pos:e])
        return "".join(out)

    def collapse(self, s, e, text):
        self.edits = [x for x in self.edits if not (x[0] >= s and x[1] <= e)]
        self.edit(s, e, text)

    # ------------------------------------------------------------------ tokens
    def peek(self, k=0):
        return self.t[min(self.i + k, len(self.t) - 1)]

    def at(self, v, k=0):
        tk = self.peek(k)
        return tk.v == v and tk.k in ("p", "id")

    def next(self):
        tk = self.t[self.i]
        self.i += 1
        return tk

    def peek_op(self):
        """Current operator, re-joining adjacent '>' tokens: returns (op, ntoks)."""
        tk = self.peek()
        if tk.k == "p" and tk.v == ">":
            ops = [">"]
            k = 1
            while len(ops) < 3:
                nx = self.peek(k)
                if nx.k == "p" and nx.s == self.peek(k - 1).e and nx.v in (">", ">="):
                    ops.append(nx.v)
                    k += 1
                    if nx.v == ">=":
                        break
                else:
                    break
            return "".join(ops), k
        return tk.v, 1

    def expect(self, v):
        tk = self.next()
        if tk.v != v:
            raise SyntaxError(f"{self.name}: expected {v!r} got {tk!r} near "
                              f"{self.src[max(0, tk.s - 80):tk.s + 40]!r}")
        return tk

    def skip_balanced(self):
        """Skip a (), [], {} or <> group starting at the current token."""
        pairs = {"(": ")", "[": "]", "{": "}", "<": ">"}
        open_ = self.next().v
        close = pairs[open_]
        depth = 1
        while depth:
            tk = self.next()
            if tk.k == "eof":
                raise SyntaxError("unbalanced")
            if tk.v == open_:
                depth += 1
            elif tk.v == close:
                depth -= 1

    # ------------------------------------------------------------------ types
    def skip_type(self):
        """Skip a type expression starting at current token.  Returns True on success."""
        if self.at("|") or self.at("&"):
            self.next()
        self.skip_type_postfix()
        while self.at("|") or self.at("&"):
            self.next()
            self.skip_type_postfix()
        if self.at("extends") and not self.peek().nl:
            # conditional type
            self.next()
            self.skip_type()
            self.expect("?")
            self.skip_type()
            self.expect(":")
            self.skip_type()
        return True

    def skip_type_postfix(self):
        self.skip_type_primary()
        while True:
            if self.at("[") and not self.peek().nl:
                self.skip_balanced()
            else:
                break

    def skip_type_primary(self):
        tk = self.peek()
        if tk.v in ("(",) and tk.k == "p":
            self.skip_balanced()
            if self.at("=>"):
                self.next()
                self.skip_type()
            return
        if tk.v == "new" and tk.k == "id":
            self.next()
            if self.at("<"):
                self.skip_balanced()
            self.skip_balanced()
            self.expect("=>")
            self.skip_type()
            return
        if tk.v == "<" and tk.k == "p":      # generic function type
            self.skip_balanced()
            self.skip_balanced()
            self.expect("=>")
            self.skip_type()
            return
        if tk.v in ("{", "[") and tk.k == "p":
            self.skip_balanced()
            return
        if tk.k == "id" and tk.v in ("typeof", "keyof", "readonly", "unique", "infer"):
            self.next()
            if tk.v == "typeof":
                self.next()
                while self.at("."):
                    self.next()
                    self.next()
                return
            self.skip_type_postfix()
            return
        if tk.k in ("str", "num", "tmpl"):
            self.next()
            return
        if tk.k == "p" and tk.v == "-":
            self.next()
            self.next()
            return
        if tk.k == "id":
            self.next()
            while self.at(".") :
                self.next()
                self.next()
            if self.at("<") and not self.peek().nl:
                self.skip_balanced()
            if self.at("is") and not self.peek().nl:
                self.next()
                self.skip_type()
            return
        raise SyntaxError(f"{self.name}: bad type token {tk!r} near {self.src[tk.s - 60:tk.s + 30]!r}")

    def try_type_args(self):
        """At '<': if it is a type-argument list (followed by '(' or valid continuation),
        consume it and return (s, e); else restore and return None."""
        save = self.i
        try:
            s = self.peek().s
            self.skip_balanced_type_args()
            e = self.t[self.i - 1].e
            nxt = self.peek()
            if nxt.v in ("(",) or (nxt.k == "tmpl"):
                return (s, e)
        except SyntaxError:
            pass
        self.i = save
        return None

    def skip_balanced_type_args(self):
        self.expect("<")
        if self.at(">"):
            raise SyntaxError("empty")
        while True:
            self.skip_type()
            if self.at(","):
                self.next()
                continue
            break
        tk = self.peek()
        if tk.v == ">":
            self.next()
        else:
            raise SyntaxError("not type args")

    # ------------------------------------------------------------------ program
    def run(self):
        while self.peek().k != "eof":
            self.statement(top=True)
        return self

    def statement(self, top=False):
        tk = self.peek()
        if tk.k == "p":
            if tk.v == "{":
                self.block()
                return
            if tk.v == ";":
                self.next()
                return
            self.expr_statement()
            return
        if tk.k != "id":
            self.expr_statement()
            return
        v = tk.v
        nx = self.peek(1)
        if v == "import" and nx.v != "(":
            self.import_decl()
            return
        if v == "export":
            self.export_decl()
            return
        if v == "interface" and nx.k == "id":
            self.skip_decl_to_block(tk.s)
            return
        if v == "type" and nx.k == "id" and self.peek(2).v in ("=", "<"):
            self.type_alias(tk.s)
            return
        if v == "declare" and nx.k == "id" and not nx.nl:
            self.declare_decl(tk.s)
            return
        if v == "namespace" and nx.k == "id":
            raise SyntaxError("namespace unsupported")
        if v == "enum" or (v == "const" and nx.v == "enum"):
            self.enum_decl(tk.s, export=False)
            return
        if v == "abstract" and nx.v == "class":
            self.next()
            self.edit(tk.s, nx.s)
            self.class_decl()
            return
        if v == "class":
            self.class_decl()
            return
        if v == "function" or (v == "async" and nx.v == "function" and not nx.nl):
            self.function_decl()
            return
        if v in ("let", "const", "var"):
            self.var_decl()
            self.semi()
            return
        if v == "if":
            self.next()
            self.paren_expr()
            self.statement()
            if self.at("else"):
                self.next()
                self.statement()
            return
        if v == "for":
            self.next()
            if self.at("await"):
                self.next()
            self.expect("(")
            if self.at("let") or self.at("const") or self.at("var"):
                self.var_decl(in_for=True)
            elif not self.at(";"):
                self.expression(no_in=True)
            if self.at("of") or self.at("in"):
                self.next()
                self.expression()
            else:
                self.expect(";")
                if not self.at(";"):
                    self.expression()
                self.expect(";")
                if not self.at(")"):
                    self.expression()
            self.expect(")")
            self.statement()
            return
        if v == "while":
            self.next()
            self.paren_expr()
            self.statement()
            return
        if v == "do":
            self.next()
            self.statement()
            self.expect("while")
            self.paren_expr()
            self.semi()
            return
        if v == "switch":
            self.next()
            self.paren_expr()
            self.expect("{")
            while not self.at("}"):
                if self.at("case"):
                    self.next()
                    self.expression()
                    self.expect(":")
                elif self.at("default"):
                    self.next()
                    self.expect(":")
                else:
                    self.statement()
            self.expect("}")
            return
        if v == "try":
            self.next()
            self.block()
            if self.at("catch"):
                self.next()
                if self.at("("):
                    self.next()
                    self.binding()
                    if self.at(":"):
                        s = self.peek().s
                        self.next()
                        self.skip_type()
                        self.edit(s, self.t[self.i - 1].e)
                    self.expect(")")
                self.block()
            if self.at("finally"):
                self.next()
                self.block()
            return
        if v in ("return", "throw"):
            self.next()
            if not self.at(";") and not self.at("}") and not self.peek().nl:
                self.expression()
            self.semi()
            return
        if v in ("break", "continue"):
            self.next()
            if self.peek().k == "id" and not self.peek().nl:
                self.next()
            self.semi()
            return
        if nx.v == ":" and nx.k == "p" and v not in ("default", "case"):
            self.next()
            self.next()
            self.statement()
            return
        self.expr_statement()

    def semi(self):
        if self.at(";"):
            self.next()

    def expr_statement(self):
        self.expression()
        self.semi()

    def block(self):
        self.expect("{")
        while not self.at("}"):
            self.statement()
        self.expect("}")

    def paren_expr(self):
        self.expect("(")
        self.expression()
        self.expect(")")

    def skip_decl_to_block(self, s):
        while not self.at("{"):
            self.next()
        self.skip_balanced()
        self.edit(s, self.t[self.i - 1].e)

    def type_alias(self, s):
        self.next()          # type
        self.next()          # name
        if self.at("<"):
            self.skip_balanced()
        self.expect("=")
        self.skip_type()
        self.semi()
        self.edit(s, self.t[self.i - 1].e)

    def declare_decl(self, s):
        self.next()
        depth = 0
        while True:
            tk = self.next()
            if tk.v in ("{", "(", "["):
                depth += 1
            elif tk.v in ("}", ")", "]"):
                depth -= 1
                if depth == 0 and tk.v == "}":
                    break
            elif tk.v == ";" and depth == 0:
                break
        self.edit(s, self.t[self.i - 1].e)

    # ------------------------------------------------------------------ modules
    def import_decl(self):
        s = self.next().s
        if self.peek().k == "str":
            mod = json.loads(self.next().v.replace("'", '"'))
            self.imports.append(("side", None, None, mod))
            self.semi()
            self.edit(s, self.t[self.i - 1].e)
            return
        specs = []
        if self.peek().k == "id" and not self.at("{") and self.peek().v != "*":
            specs.append(("default", self.next().v, "default"))
            if self.at(","):
                self.next()
        if self.at("*"):
            self.next()
            self.expect("as")
            specs.append(("ns", self.next().v, "*"))
        elif self.at("{"):
            self.next()
            while not self.at("}"):
                imported = self.next().v
                local = imported
                if self.at("as"):
                    self.next()
                    local = self.next().v
                specs.append(("named", local, imported))
                if self.at(","):
                    self.next()
            self.expect("}")
        self.expect("from")
        mod = json.loads(self.next().v.replace("'", '"'))
        self.semi()
        for kind, local, imported in specs:
            self.imports.append((kind, local, imported, mod))
        self.edit(s, self.t[self.i - 1].e)

    def export_decl(self):
        ex = self.next()
        tk = self.peek()
        v = tk.v
        if v in ("interface",) or (v == "type" and self.peek(1).k == "id"
                                   and self.peek(2).v in ("=", "<")):
            if v == "interface":
                self.skip_decl_to_block(ex.s)
            else:
                self.type_alias(ex.s)
            return
        if v == "declare":
            self.declare_decl(ex.s)
            return
        if v == "default":
            self.next()
            if self.at("class"):
                self.class_decl()
            elif self.at("function"):
                self.function_decl()
            else:
                self.expression()
                self.semi()
            self.exported.add("default")
            return
        if v == "*":
            self.next()
            self.expect("from")
            mod = json.loads(self.next().v.replace("'", '"'))
            self.semi()
            self.reexports.append(("*", None, mod))
            self.edit(ex.s, self.t[self.i - 1].e)
            return
        if v == "{":
            self.next()
            names = []
            while not self.at("}"):
                local = self.next().v
                exported = local
                if self.at("as"):
                    self.next()
                    exported = self.next().v
                names.append((local, exported))
                if self.at(","):
                    self.next()
            self.expect("}")
            mod = None
            if self.at("from"):
                self.next()
                mod = json.loads(self.next().v.replace("'", '"'))
            self.semi()
            self.reexports.append(("names", names, mod))
            self.edit(ex.s, self.t[self.i - 1].e)
            return
        if v == "enum" or (v == "const" and self.peek(1).v == "enum"):
            self.enum_decl(ex.s, export=True)
            return
        if v == "abstract":
            self.edit(tk.s, self.peek(1).s)
            self.next()
        if self.at("class"):
            name = self.peek(1).v
            self.exported.add(name)
            self.class_decl()
            return
        if self.at("function") or self.at("async"):
            nm = self.peek(1).v if self.at("function") else self.peek(2).v
            if nm == "*":
                nm = self.peek(2).v
            self.exported.add(nm)
            self.function_decl()
            return
        if v in ("let", "const", "var"):
            names = self.var_decl()
            self.exported.update(names)
            self.semi()
            return
        raise SyntaxError(f"{self.name}: unsupported export {tk!r}")

    # ------------------------------------------------------------------ enums
    def enum_decl(self, s, export):
        if self.at("const"):
            self.next()
        self.expect("enum")
        name = self.next().v
        self.expect("{")
        members = []
        while not self.at("}"):
            mtk = self.next()
            mname = json.loads(mtk.v) if mtk.k == "str" else mtk.v
            init = None
            if self.at("="):
                self.next()
                es = self.peek().s
                self.assign_expr()
                init = self.render(es, self.t[self.i - 1].e)
            members.append((mname, init))
            if self.at(","):
                self.next()
        self.expect("}")
        e = self.t[self.i - 1].e
        lines = [f"{'export ' if export else ''}var {name};", f"(function ({name}) {{"]
        auto = 0
        names = {m for m, _ in members}
        for mname, init in members:
            if init is None:
                val = str(auto)
                auto += 1
                lines.append(f"    {name}[{name}[{json.dumps(mname)}] = {val}] = {json.dumps(mname)};")
            else:
                # resolve bare references to earlier members
                expr = re.sub(r"\b([A-Za-z_$][\w$]*)\b",
                              lambda m: f"{name}.{m.group(1)}" if m.group(1) in names else m.group(1),
                              init)
                if init.strip().startswith(("'", '"')):
                    lines.append(f"    {name}[{json.dumps(mname)}] = {expr};")
                else:
                    lines.append(f"    {name}[{name}[{json.dumps(mname)}] = {expr}] = {json.dumps(mname)};")
                    try:
                        auto = int(eval(init.replace("0x", "0x"), {})) + 1
                    except Exception:
                        auto = None
        lines.append(f"}})({name} || ({name} = {{}}));")
        self.collapse(s, e, "\n".join(lines))
        if export:
            self.exported.add(name)

    # ------------------------------------------------------------------ declarations
    def var_decl(self, in_for=False):
        self.next()      # let/const/var
        names = []
        while True:
            names.extend(self.binding())
            if self.at("!"):
                t = self.next()
                self.edit(t.s, t.e)
            if self.at(":"):
                s = self.peek().s
                self.next()
                self.skip_type()
                self.edit(s, self.t[self.i - 1].e)
            if self.at("="):
                self.next()
                self.assign_expr(no_in=in_for)
            if self.at(","):
                self.next()
                continue
            break
        return names

    def binding(self):
        """Binding identifier or pattern; returns bound names (top-level only)."""
        tk = self.peek()
        if tk.v in ("{", "[") and tk.k == "p":
            close = "}" if tk.v == "{" else "]"
            self.next()
            names = []
            while not self.at(close):
                if self.at(","):
                    self.next()
                    continue
                if self.at("..."):
                    self.next()
                if tk.v == "{":
                    key = self.next()
                    if self.at(":"):
                        self.next()
                        names.extend(self.binding())
                    else:
                        names.append(key.v)
                else:
                    names.extend(self.binding())
                if self.at("="):
                    self.next()
                    self.assign_expr()
                if self.at(","):
                    self.next()
            self.expect(close)
            return names
        return [self.next().v]

    def function_decl(self):
        if self.at("async"):
            self.next()
        self.expect("function")
        if self.at("*"):
            self.next()
        if self.peek().k == "id" and not self.at("("):
            self.next()
        self.function_rest(allow_overload=True, decl_start=None)

    def function_rest(self, allow_overload=False, decl_start=None, is_ctor=False):
        """At optional <T> then params.  Returns (param_props, body_open_tok or None)."""
        if self.at("<"):
            s = self.peek().s
            self.skip_balanced()
            self.edit(s, self.t[self.i - 1].e)
        pprops = self.params()
        if self.at(":"):
            s = self.peek().s
            self.next()
            self.skip_type()
            self.edit(s, self.t[self.i - 1].e)
        if self.at("{"):
            open_tok = self.peek()
            body = self.fn_body()
            return pprops, open_tok, body
        # overload / abstract signature
        self.semi()
        return pprops, None, None

    def fn_body(self):
        """Parse a function body; return list of (stmt_start_idx, stmt_end_idx) for top statements."""
        self.expect("{")
        stmts = []
        while not self.at("}"):
            si = self.i
            self.statement()
            stmts.append((si, self.i))
        self.expect("}")
        return stmts

    def params(self):
        self.expect("(")
        pprops = []
        first = True
        while not self.at(")"):
            ps = self.peek().s
            mods = []
            while self.peek().k == "id" and self.peek().v in ("public", "private", "protected",
                                                               "readonly", "override") \
                    and self.peek(1).k in ("id",) or (self.peek().v in ("public", "private", "protected", "readonly")
                                                      and self.peek(1).v in ("{", "[")):
                mt = self.next()
                mods.append(mt)
            if mods:
                self.edit(mods[0].s, self.peek().s)
            if first and self.at("this") and self.peek(1).v == ":":
                # TS `this` parameter
                s = self.peek().s
                self.next()
                self.next()
                self.skip_type()
                if self.at(","):
                    self.next()
                self.edit(s, self.peek().s)
                first = False
                continue
            first = False
            if self.at("..."):
                self.next()
            names = self.binding()
            if self.at("?"):
                t = self.next()
                self.edit(t.s, t.e)
            if self.at(":"):
                s = self.peek().s
                self.next()
                self.skip_type()
                self.edit(s, self.t[self.i - 1].e)
            if self.at("="):
                self.next()
                self.assign_expr()
            if mods:
                pprops.extend(names)
            if self.at(","):
                self.next()
        self.expect(")")
        return pprops

    # ------------------------------------------------------------------ classes
    def class_decl(self):
        ctk = self.expect("class")
        name = None
        if self.peek().k == "id" and not self.at("extends") and not self.at("implements") \
                and not self.at("{"):
            name = self.next().v
        if self.at("<"):
            s = self.peek().s
            self.skip_balanced()
            self.edit(s, self.t[self.i - 1].e)
        derived = False
        if self.at("extends"):
            derived = True
            self.next()
            self.lhs_expr()
            if self.at("<"):
                s = self.peek().s
                self.skip_balanced()
                self.edit(s, self.t[self.i - 1].e)
        if self.at("implements"):
            s = self.peek().s
            self.next()
            self.skip_type()
            while self.at(","):
                self.next()
                self.skip_type()
            self.edit(s, self.t[self.i - 1].e)
        self.class_body(derived)
        return name

    def class_body(self, derived):
        self.expect("{")
        fields = []          # rendered "this.x = init;" strings in order
        ctor = None          # (pprops, body_open_tok, stmts)
        while not self.at("}"):
            if self.at(";"):
                self.next()
                continue
            ms = self.peek().s
            mods = []
            while self.peek().k == "id" and self.peek().v in MODIFIERS | {"get", "set"} \
                    and self.peek(1).v not in ("(", "=", ";", ":", "?", "!", "<") \
                    and not self.peek(1).nl:
                mods.append(self.next())
            # decide kind
            modnames = {m.v for m in mods}
            for m in mods:
                if m.v in ("public", "private", "protected", "readonly", "override", "declare"):
                    self.edit(m.s, self.peek().s if m is mods[-1] else mods[mods.index(m) + 1].s)
            if self.at("["):
                # index signature or computed name
                save = self.i
                self.next()
                if self.peek().k == "id" and self.peek(1).v == ":":
                    self.i = save
                    self.skip_balanced()
                    if self.at(":"):
                        self.next()
                        self.skip_type()
                    self.semi()
                    self.edit(ms, self.t[self.i - 1].e)
                    continue
                self.i = save
                self.skip_balanced()
                name_tok = None
            else:
                if self.at("*"):
                    self.next()
                name_tok = self.next()
            if self.at("?") or self.at("!"):
                t = self.next()
                self.edit(t.s, t.e)
            if self.at("(") or self.at("<"):
                is_ctor = name_tok is not None and name_tok.v == "constructor"
                pprops, body_open, stmts = self.function_rest(is_ctor=is_ctor)
                if body_open is None:
                    # abstract method or overload signature
                    self.collapse(ms, self.t[self.i - 1].e, "")
                    continue
                if is_ctor:
                    ctor = (pprops, body_open, stmts)
                continue
            # property
            init = None
            if self.at(":"):
                s = self.peek().s
                self.next()
                self.skip_type()
                self.edit(s, self.t[self.i - 1].e)
            if self.at("="):
                self.next()
                es = self.peek().s
                self.assign_expr()
                init = (es, self.t[self.i - 1].e)
            self.semi()
            me = self.t[self.i - 1].e
            if "abstract" in modnames or "declare" in modnames:
                self.collapse(ms, me, "")
                continue
            if "static" in modnames:
                if init is None:
                    self.collapse(ms, me, "")
                continue
            if init is None:
                self.collapse(ms, me, "")
            else:
                prop = name_tok.v if name_tok is not None else None
                key = f"this.{prop}" if name_tok.k == "id" else f"this[{prop}]"
                fields.append(f"{key} = {self.render(*init)};")
                self.collapse(ms, me, "")
        close = self.expect("}")
        # constructor synthesis
        if ctor is None:
            if fields:
                if derived:
                    text = "constructor(...args) { super(...args); " + " ".join(fields) + " }\n"
                else:
                    text = "constructor() { " + " ".join(fields) + " }\n"
                self.edit(close.s, close.s, text)
            return
        pprops, body_open, stmts = ctor
        assigns = [f"this.{p} = {p};" for p in pprops] + fields
        if not assigns:
            return
        text = " " + " ".join(assigns) + " "
        pos = body_open.e
        if derived:
            for si, ei in stmts:
                tk0 = self.t[si]
                if tk0.v == "super" and self.t[si + 1].v == "(":
                    pos = self.t[ei - 1].e
                    break
        self.edit(pos, pos, text)

    # ------------------------------------------------------------------ expressions
    def expression(self, no_in=False):
        self.assign_expr(no_in)
        while self.at(","):
            self.next()
            self.assign_expr(no_in)

    def is_arrow_at_paren(self):
        save = self.i
        try:
            self.skip_balanced()
            if self.at("=>") and not self.peek().nl:
                return True
            if self.at(":"):
                self.next()
                self.skip_type()
                return self.at("=>")
            return False
        except SyntaxError:
            return False
        finally:
            self.i = save

    def arrow(self):
        """At params of an arrow function (ident or '(')."""
        if self.at("async") and (self.peek(1).k == "id" or self.peek(1).v == "("):
            self.next()
        if self.at("("):
            self.params()
            if self.at(":"):
                s = self.peek().s
                self.next()
                self.skip_type()
                self.edit(s, self.t[self.i - 1].e)
        else:
            self.next()
        self.expect("=>")
        if self.at("{"):
            self.fn_body()
        else:
            self.assign_expr()

    def assign_expr(self, no_in=False):
        tk = self.peek()
        if tk.k == "id" and self.peek(1).v == "=>" and tk.v not in ("this",):
            self.arrow()
            return
        if tk.k == "id" and tk.v == "async" and not self.peek(1).nl and (
                (self.peek(1).k == "id" and self.peek(2).v == "=>") or
                (self.peek(1).v == "(" and self._arrow_after(1))):
            self.arrow()
            return
        if tk.v == "(" and tk.k == "p" and self.is_arrow_at_paren():
            self.arrow()
            return
        if tk.v == "<" and tk.k == "p":
            # generic arrow  <T>(x: T) => ...
            save = self.i
            try:
                s = tk.s
                self.skip_balanced()
                if self.at("(") and self.is_arrow_at_paren():
                    self.edit(s, self.t[self.i - 1].e)
                    self.arrow()
                    return
            except SyntaxError:
                pass
            self.i = save
        if tk.k == "id" and tk.v == "yield":
            self.next()
            if not self.at(")") and not self.at(";") and not self.at(","):
                self.assign_expr(no_in)
            return
        self.conditional(no_in)
        op, n = self.peek_op()
        if op in ASSIGN_OPS and self.peek().k == "p":
            self.i += n
            self.assign_expr(no_in)

    def _arrow_after(self, k):
        save = self.i
        self.i += k
        r = self.is_arrow_at_paren()
        self.i = save
        return r

    def conditional(self, no_in=False):
        self.binary(0, no_in)
        if self.at("?"):
            self.next()
            self.assign_expr()
            self.expect(":")
            self.assign_expr(no_in)

    def binary(self, minprec, no_in=False):
        ls = self.peek().s
        self.unary()
        while True:
            tk = self.peek()
            op, nt = self.peek_op()
            if tk.k not in ("p", "id") or op not in BIN_PREC:
                break
            if tk.k == "id" and op not in ("instanceof", "in", "as"):
                break
            if op == "in" and no_in:
                break
            if op == "as":
                if tk.nl:
                    break
                self.next()
                if self.at("const"):
                    self.next()
                else:
                    self.skip_type()
                self.edit(tk.s, self.t[self.i - 1].e)
                continue
            prec = BIN_PREC[op]
            if prec < minprec:
                break
            self.i += nt
            rs = self.peek().s
            self.binary(prec + (0 if op == "**" else 1), no_in)
            re_ = self.t[self.i - 1].e
            if op == "??":
                left = self.render(ls, tk.s).strip()
                right = self.render(rs, re_).strip()
                self.collapse(ls, re_, f"(({left}) != null ? ({left}) : ({right}))")

    def unary(self):
        tk = self.peek()
        if tk.k == "p" and tk.v in ("!", "-", "+", "~", "++", "--"):
            self.next()
            self.unary()
            return
        if tk.k == "id" and tk.v in ("typeof", "void", "delete", "await") and \
                not (self.peek(1).k == "p" and self.peek(1).v in (")", ",", ";", "=", ".", "=>")):
            self.next()
            self.unary()
            return
        if tk.k == "p" and tk.v == "<":
            # type assertion <T>expr
            s = tk.s
            self.skip_balanced()
            self.edit(s, self.t[self.i - 1].e, "(")
            self.unary()
            e = self.t[self.i - 1].e
            self.edit(e, e, ")")
            return
        self.postfix()

    def lhs_expr(self):
        self.postfix()

    def postfix(self):
        s = self.peek().s
        self.primary()
        parts = []      # (optional, start, end)
        has_opt = False
        while True:
            tk = self.peek()
            if tk.k == "p" and tk.v == ".":
                ps = tk.s
                self.next()
                self.next()
                parts.append((False, ps, self.t[self.i - 1].e))
            elif tk.k == "p" and tk.v == "?.":
                has_opt = True
                ps = tk.s
                self.next()
                if self.at("("):
                    self.args()
                elif self.at("["):
                    self.next()
                    self.expression()
                    self.expect("]")
                else:
                    self.next()
                parts.append((True, ps, self.t[self.i - 1].e))
            elif tk.k == "p" and tk.v == "[" :
                ps = tk.s
                self.next()
                self.expression()
                self.expect("]")
                parts.append((False, ps, self.t[self.i - 1].e))
            elif tk.k == "p" and tk.v == "(":
                ps = tk.s
                self.args()
                parts.append((False, ps, self.t[self.i - 1].e))
            elif tk.k == "tmpl":
                self.next()
                parts.append((False, tk.s, tk.e))
            elif tk.k == "p" and tk.v == "!" and not tk.nl:
                nxt = self.peek(1)
                if nxt.k == "p" and nxt.v in (".", ")", ",", ";", "]", "[", "(", "}", ":", "=", "?.") \
                        or nxt.k == "eof" or nxt.nl or (nxt.k == "id" and nxt.v in ("as",)):
                    self.next()
                    self.edit(tk.s, tk.e)
                    parts.append((False, tk.s, tk.e))
                else:
                    break
            elif tk.k == "p" and tk.v == "<" and not tk.nl:
                ta = self.try_type_args()
                if ta is None:
                    break
                self.edit(*ta)
                parts.append((False, ta[0], ta[1]))
            elif tk.k == "p" and tk.v in ("++", "--") and not tk.nl:
                self.next()
                break
            else:
                break
        if has_opt:
            base_end = parts[0][1]
            cur = self.render(s, base_end)
            pieces = [(o, self.render(a, b)) for o, a, b in parts]

            def build(cur, pieces):
                for idx, (opt, txt) in enumerate(pieces):
                    if opt:
                        t2 = txt[2:]
                        if not t2.startswith(("(", "[")):
                            t2 = "." + t2
                        return f"({cur} == null ? undefined : {build(cur + t2, pieces[idx + 1:])})"
                    cur += txt
                return cur
            self.collapse(s, self.t[self.i - 1].e, build(cur, pieces))

    def args(self):
        self.expect("(")
        while not self.at(")"):
            if self.at("..."):
                self.next()
            self.assign_expr()
            if self.at(","):
                self.next()
        self.expect(")")

    def primary(self):
        tk = self.peek()
        if tk.k in ("num", "str", "tmpl", "re"):
            self.next()
            return
        if tk.k == "p":
            if tk.v == "(":
                self.next()
                self.expression()
                self.expect(")")
                return
            if tk.v == "[":
                self.next()
                while not self.at("]"):
                    if self.at(","):
                        self.next()
                        continue
                    if self.at("..."):
                        self.next()
                    self.assign_expr()
                    if self.at(","):
                        self.next()
                self.expect("]")
                return
            if tk.v == "{":
                self.object_literal()
                return
            if tk.v == "#":
                self.next()
                self.next()
                return
            raise SyntaxError(f"{self.name}: unexpected {tk!r} near {self.src[tk.s - 80:tk.s + 40]!r}")
        if tk.k == "id":
            v = tk.v
            if v == "function" or (v == "async" and self.peek(1).v == "function"):
                if v == "async":
                    self.next()
                self.next()
                if self.at("*"):
                    self.next()
                if self.peek().k == "id":
                    self.next()
                self.function_rest()
                return
            if v == "class":
                self.class_decl()
                return
            if v == "new":
                self.next()
                if self.at("."):
                    self.next()
                    self.next()
                    return
                # new Callee<T>(args)
                s = self.peek().s
                self.primary()
                while self.at(".") or self.at("["):
                    if self.at("."):
                        self.next()
                        self.next()
                    else:
                        self.next()
                        self.expression()
                        self.expect("]")
                if self.at("<"):
                    ta = self.try_type_args()
                    if ta is not None:
                        self.edit(*ta)
                    else:
                        st = self.peek().s
                        self.skip_balanced()
                        self.edit(st, self.t[self.i - 1].e)
                if self.at("("):
                    self.args()
                return
            self.next()
            return
        raise SyntaxError(f"unexpected {tk!r}")

    def object_literal(self):
        self.expect("{")
        while not self.at("}"):
            if self.at("..."):
                self.next()
                self.assign_expr()
            else:
                tk = self.peek()
                is_acc = tk.k == "id" and tk.v in ("get", "set", "async") and \
                    self.peek(1).v not in (",", ":", "(", "}")
                if is_acc:
                    self.next()
                if self.at("*"):
                    self.next()
                if self.at("["):
                    self.next()
                    self.assign_expr()
                    self.expect("]")
                else:
                    self.next()
                if self.at("(") or self.at("<"):
                    self.function_rest()
                elif self.at(":"):
                    self.next()
                    self.assign_expr()
                elif self.at("="):
                    self.next()
                    self.assign_expr()
            if self.at(","):
                self.next()
            elif not self.at("}"):
                tk = self.peek()
                raise SyntaxError(f"{self.name}: object literal near {self.src[tk.s - 80:tk.s + 40]!r}")
        self.expect("}")


# ---------------------------------------------------------------------- driver
IDENT_RE = re.compile(r"[A-Za-z_$][\w$]*")


def used_identifiers(js):
    """Identifiers appearing in value positions of the rendered JS (approximate)."""
    used = set()
    for tk in lex(js):
        pass
    toks = lex(js)
    for k, tk in enumerate(toks):
        if tk.k != "id":
            continue
        prev = toks[k - 1] if k else None
        if prev is not None and prev.k == "p" and prev.v in (".", "?."):
            continue
        nxt = toks[k + 1]
        # object literal key  { name: value }  (not shorthand)
        if nxt.k == "p" and nxt.v == ":" and prev is not None and prev.v in ("{", ","):
            continue
        used.add(tk.v)
    return used


def transpile_tree(files, resolve_module):
    """files: dict modname -> (path, src).  Returns dict modname -> js text.

    resolve_module(from_mod, spec) -> target modname (in files) or ("shim", path)."""
    units = {}
    for mod, (path, src) in files.items():
        try:
            units[mod] = Transpiler(src, path).run()
        except Exception as exc:
            raise RuntimeError(f"transpile failed in {path}: {exc}") from exc

    # value exports per module (transitive through export *)
    local_exports = {m: set(u.exported) for m, u in units.items()}
    for m, u in units.items():
        for kind, names, mod in u.reexports:
            if kind == "names" and mod is None:
                local_exports[m].update(e for _, e in names)
    value_exports = {}

    def vexp(m, stack=()):
        if m in value_exports:
            return value_exports[m]
        if m not in units:
            return None        # shim: accept everything
        if m in stack:
            return set()
        res = set(local_exports[m])
        for kind, names, mod in units[m].reexports:
            tgt = resolve_module(m, mod) if mod else None
            if kind == "*":
                sub = vexp(tgt, stack + (m,)) if isinstance(tgt, str) else None
                if sub is not None:
                    res |= sub - {"default"}
            elif kind == "names" and mod is not None:
                sub = vexp(tgt, stack + (m,)) if isinstance(tgt, str) else None
                for local, exported in names:
                    if sub is None or local in sub:
                        res.add(exported)
        value_exports[m] = res
        return res

    for m in units:
        vexp(m)

    out = {}
    for m, u in units.items():
        body = u.render(0, len(u.src))
        used = used_identifiers(body)
        header = []
        by_mod = {}
        for kind, local, imported, mod in u.imports:
            by_mod.setdefault(mod, []).append((kind, local, imported))
        for mod, specs in by_mod.items():
            tgt = resolve_module(m, mod)
            spec_path = tgt[1] if isinstance(tgt, tuple) else "./" + tgt + ".mjs"
            if isinstance(tgt, str):
                spec_path = os.path.relpath(tgt, os.path.dirname(m) or ".") + ".mjs"
                if not spec_path.startswith("."):
                    spec_path = "./" + spec_path
            tvals = value_exports.get(tgt) if isinstance(tgt, str) else None
            default = [l for k, l, i in specs if k == "default" and l in used]
            ns = [l for k, l, i in specs if k == "ns" and l in used]
            named = [(l, i) for k, l, i in specs if k == "named" and l in used
                     and (tvals is None or i in tvals)]
            side = any(k == "side" for k, l, i in specs)
            for l in ns:
                header.append(f"import * as {l} from {json.dumps(spec_path)};")
            parts = []
            if default:
                parts.append(default[0])
            if named:
                parts.append("{ " + ", ".join(i if i == l else f"{i} as {l}" for l, i in named) + " }")
            if parts:
                header.append(f"import {', '.join(parts)} from {json.dumps(spec_path)};")
            elif side and not ns:
                header.append(f"import {json.dumps(spec_path)};")
        footer = []
        for kind, names, mod in u.reexports:
            if kind == "*":
                tgt = resolve_module(m, mod)
                p = os.path.relpath(tgt, os.path.dirname(m) or ".") + ".mjs" if isinstance(tgt, str) else tgt[1]
                if not p.startswith(".") and not p.startswith("/"):
                    p = "./" + p
                footer.append(f"export * from {json.dumps(p)};")
            else:
                if mod is None:
                    keep = [(l, e) for l, e in names if l in used or l in local_exports[m]
                            or any(l == x[1] for x in u.imports)]
                    keep = [(l, e) for l, e in keep if _is_value_local(u, l, value_exports, resolve_module, m)]
                    if keep:
                        footer.append("export { " + ", ".join(l if l == e else f"{l} as {e}" for l, e in keep) + " };")
                else:
                    tgt = resolve_module(m, mod)
                    p = os.path.relpath(tgt, os.path.dirname(m) or ".") + ".mjs" if isinstance(tgt, str) else tgt[1]
                    if not p.startswith(".") and not p.startswith("/"):
                        p = "./" + p
                    tvals = value_exports.get(tgt) if isinstance(tgt, str) else None
                    keep = [(l, e) for l, e in names if tvals is None or l in tvals]
                    if keep:
                        footer.append("export { " + ", ".join(l if l == e else f"{l} as {e}" for l, e in keep)
                                      + f" }} from {json.dumps(p)};")
        out[m] = "\n".join(header) + "\n" + body + "\n" + "\n".join(footer) + "\n"
    return out


def _is_value_local(u, name, value_exports, resolve_module, m):
    if name in u.exported:
        return True
    for kind, local, imported, mod in u.imports:
        if local == name:
            tgt = resolve_module(m, mod)
            tv = value_exports.get(tgt) if isinstance(tgt, str) else None
            return tv is None or imported in tv or kind == "ns"
    # local declaration (class/function/const) not exported directly
    return re.search(r"\b(class|function|const|let|var)\s+" + re.escape(name) + r"\b", u.src) is not None


if __name__ == "__main__":
    src = open(sys.argv[1]).read()
    u = Transpiler(src, sys.argv[1]).run()
    sys.stdout.write(u.render(0, len(src)))
