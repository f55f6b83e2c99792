"""A small renderer for this repo's helm chart (no helm binary in the image).

Implements the subset of Go text/template + sprig the chart uses: actions with
`{{-`/`-}}` whitespace trimming, comments, pipelines, parenthesised commands,
variables (`$x :=`), `if`/`else if`/`else`, `with`/`else`, `define`/`include`,
`.Files.Get`, and the functions default, kindIs, trunc, trimSuffix, contains, printf, toYaml,
nindent, indent, quote, replace, coalesce, or, and, not, eq. Enough to render
deployments/helm/amd-gpu-device-plugin for tests/test_helm_render.py; it is
not a general helm implementation.

    python tools/helm_render.py [--set key=value ...] > daemonset.yaml
"""

import copy
import os
import re
import sys

import yaml

CHART = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                     "deployments", "helm", "amd-gpu-device-plugin")


# ---- lexing ---------------------------------------------------------------

def _lex(src):
    """[("text", s) | ("action", body)] with trim markers applied."""
    out, pos = [], 0
    while True:
        i = src.find("{{", pos)
        if i < 0:
            out.append(["text", src[pos:]])
            return out
        j = src.find("}}", i)
        if j < 0:
            raise SyntaxError("unclosed action")
        body = src[i + 2:j]
        ltrim = body.startswith("-") and (len(body) > 1 and body[1] in " \t\n")
        rtrim = body.endswith("-") and (len(body) > 1 and body[-2] in " \t\n")
        text = src[pos:i]
        if ltrim:
            text = text.rstrip(" \t\r\n")
        out.append(["text", text])
        body = body[1:] if ltrim else body
        body = body[:-1] if rtrim else body
        out.append(["action", body.strip()])
        pos = j + 2
        if rtrim:
            while pos < len(src) and src[pos] in " \t\r\n":
                pos += 1


_TOKEN = re.compile(r'\s*(?:(?P<str>"(?:[^"\\]|\\.)*")|(?P<num>-?\d+(?:\.\d+)?)|(?P<assign>:=)|(?P<pipe>\|)'
                    r'|(?P<lp>\()|(?P<rp>\))|(?P<var>\$[A-Za-z0-9_]*(?:\.[A-Za-z0-9_]+)*)'
                    r'|(?P<field>\.[A-Za-z0-9_.]*)|(?P<ident>[A-Za-z_][A-Za-z0-9_]*))')


def _tokens(s):
    out, pos = [], 0
    s = s.strip()
    while pos < len(s):
        m = _TOKEN.match(s, pos)
        if not m or m.end() == pos:
            raise SyntaxError(f"cannot tokenise {s[pos:]!r}")
        kind = m.lastgroup
        out.append((kind, m.group(kind)))
        pos = m.end()
        while pos < len(s) and s[pos].isspace():
            pos += 1
    return out


# ---- parsing --------------------------------------------------------------

def _parse_pipeline(toks):
    """Pipeline = [commands]; command = [args]; arg = token or ("sub", pipeline)."""
    assign = None
    if len(toks) >= 2 and toks[0][0] == "var" and toks[1][0] == "assign":
        assign, toks = toks[0][1], toks[2:]
    cmds, cur, depth, sub = [], [], 0, []
    for t in toks:
        if depth:
            if t[0] == "lp":
                depth += 1
            elif t[0] == "rp":
                depth -= 1
                if depth == 0:
                    cur.append(("sub", _parse_pipeline(sub)))
                    sub = []
                    continue
            sub.append(t)
        elif t[0] == "lp":
            depth = 1
        elif t[0] == "pipe":
            cmds.append(cur)
            cur = []
        else:
            cur.append(t)
    cmds.append(cur)
    return {"assign": assign, "cmds": cmds}


def _parse(items, i=0, stop=()):
    """Returns (nodes, index, stop keyword hit, its action body)."""
    nodes = []
    while i < len(items):
        kind, val = items[i]
        i += 1
        if kind == "text":
            if val:
                nodes.append(("text", val))
            continue
        if val.startswith("/*"):
            continue
        word = val.split(None, 1)[0] if val else ""
        rest = val[len(word):].strip()
        if word in stop:
            return nodes, i, word, rest
        if word == "if" or word == "with":
            branches, els = [], None
            cond = rest
            while True:
                body, i, hit, hrest = _parse(items, i, ("else", "end"))
                branches.append((cond, body))
                if hit == "end":
                    break
                if hrest.startswith("if "):
                    cond = hrest[3:]
                    continue
                els, i, hit, _ = _parse(items, i, ("end",))
                break
            nodes.append((word, [(_parse_pipeline(_tokens(c)), b) for c, b in branches], els))
        elif word == "define":
            name = yaml.safe_load(rest)
            body, i, _, _ = _parse(items, i, ("end",))
            nodes.append(("define", name, body))
        else:
            nodes.append(("action", _parse_pipeline(_tokens(val))))
    return nodes, i, None, None


# ---- evaluation -----------------------------------------------------------

def gostr(v):
    if v is None:
        return ""
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, float) and v.is_integer():
        return str(int(v))
    return str(v)


def truthy(v):
    return not (v is None or v is False or v == 0 and not isinstance(v, bool) or v in ("", [], {}))


def _printf(fmt, *args):
    out, ai = [], 0
    for piece in re.split(r"(%[sdvq])", fmt):
        if re.fullmatch(r"%[sdvq]", piece):
            a = args[ai]
            ai += 1
            out.append('"%s"' % gostr(a) if piece == "%q" else gostr(a))
        else:
            out.append(piece)
    return "".join(out)


def _to_yaml(v):
    if v is None or v == {} or v == []:
        return "{}" if isinstance(v, dict) else ("[]" if isinstance(v, list) else "null")
    return yaml.safe_dump(v, default_flow_style=False, sort_keys=True).rstrip("\n")


def _kind_is(kind, v):
    """sprig kindIs: the Go reflect kind of a values-file value."""
    kinds = {"invalid": v is None, "bool": isinstance(v, bool), "string": isinstance(v, str),
             "map": isinstance(v, dict), "slice": isinstance(v, list),
             "int64": isinstance(v, int) and not isinstance(v, bool), "float64": isinstance(v, float)}
    return kinds.get(kind, False)


class Renderer:
    def __init__(self, values, chart, release):
        self.defines = {}
        self.root = {"Values": values, "Chart": chart, "Release": release}
        self.funcs = {
            "default": lambda d, v=None: v if truthy(v) else d,
            "trunc": lambda n, s: gostr(s)[:n],
            "trimSuffix": lambda suf, s: gostr(s)[:-len(suf)] if suf and gostr(s).endswith(suf) else gostr(s),
            "contains": lambda sub, s: gostr(sub) in gostr(s),
            "hasPrefix": lambda pre, s: gostr(s).startswith(gostr(pre)),
            "toString": lambda v: gostr(v),
            "printf": _printf,
            "toYaml": _to_yaml,
            "nindent": lambda n, s: "\n" + "\n".join((" " * n + ln) if ln else ln for ln in gostr(s).split("\n")),
            "indent": lambda n, s: "\n".join((" " * n + ln) if ln else ln for ln in gostr(s).split("\n")),
            "quote": lambda *a: " ".join('"%s"' % gostr(x).replace('"', '\\"') for x in a),
            "replace": lambda old, new, s: gostr(s).replace(old, new),
            "coalesce": lambda *a: next((x for x in a if truthy(x)), None),
            "or": lambda *a: next((x for x in a if truthy(x)), a[-1] if a else None),
            "and": lambda *a: next((x for x in a if not truthy(x)), a[-1] if a else None),
            "not": lambda x: not truthy(x),
            "eq": lambda a, b: a == b,
            "kindIs": _kind_is,
            "include": self._include,
        }

    def _include(self, name, dot):
        return self.render_nodes(self.defines[name], dot, {})

    def lookup(self, path, base):
        v = base
        for part in [p for p in path.split(".") if p]:
            if isinstance(v, dict):
                v = v.get(part)
            else:
                return None
        return v

    def arg(self, t, dot, scope):
        kind, val = t
        if kind == "sub":
            return self.pipeline(val, dot, scope)
        if kind == "str":
            return bytes(val[1:-1], "utf-8").decode("unicode_escape")
        if kind == "num":
            return float(val) if "." in val else int(val)
        if kind == "field":
            return dot if val == "." else self.lookup(val, dot)
        if kind == "var":
            name, _, path = val.partition(".")
            base = self.root if name == "$" else scope[name]
            return self.lookup(path, base) if path else base
        if kind == "ident":
            if val in ("true", "false"):
                return val == "true"
            if val == "nil":
                return None
            return self.funcs[val]()
        raise SyntaxError(f"bad argument {t}")

    def command(self, cmd, dot, scope, piped=None, has_piped=False):
        head = cmd[0]
        if head[0] == "ident" and head[1] in self.funcs:
            args = [self.arg(t, dot, scope) for t in cmd[1:]]
            if has_piped:
                args.append(piped)
            return self.funcs[head[1]](*args)
        if head[0] == "field" and len(cmd) > 1:  # a method, e.g. .Files.Get "path"
            fn = self.arg(head, dot, scope)
            if callable(fn):
                args = [self.arg(t, dot, scope) for t in cmd[1:]]
                return fn(*(args + [piped] if has_piped else args))
        if len(cmd) != 1 or has_piped:
            raise SyntaxError(f"not a function: {cmd}")
        return self.arg(head, dot, scope)

    def pipeline(self, p, dot, scope):
        val, has = None, False
        for cmd in p["cmds"]:
            val = self.command(cmd, dot, scope, val, has)
            has = True
        if p["assign"]:
            scope[p["assign"]] = val
            return None
        return val

    def render_nodes(self, nodes, dot, scope):
        out = []
        for n in nodes:
            kind = n[0]
            if kind == "text":
                out.append(n[1])
            elif kind == "action":
                v = self.pipeline(n[1], dot, scope)
                if not n[1]["assign"]:
                    out.append(gostr(v))
            elif kind == "define":
                self.defines[n[1]] = n[2]
            elif kind in ("if", "with"):
                for cond, body in n[1]:
                    v = self.pipeline(cond, dot, scope)
                    if truthy(v):
                        out.append(self.render_nodes(body, v if kind == "with" else dot, dict(scope)))
                        break
                else:
                    if n[2] is not None:
                        out.append(self.render_nodes(n[2], dot, dict(scope)))
        return "".join(out)

    def load(self, text):
        nodes, _, _, _ = _parse(_lex(text))
        return nodes


def merge(dst, src):
    for k, v in src.items():
        if isinstance(v, dict) and isinstance(dst.get(k), dict):
            merge(dst[k], v)
        else:
            dst[k] = v
    return dst


def render(values_override=None, release="amdgpu", chart_dir=CHART, notes=False):
    """Renders every template of the chart; returns {template file: text}."""
    with open(os.path.join(chart_dir, "values.yaml")) as f:
        values = yaml.safe_load(f)
    merge(values, copy.deepcopy(values_override or {}))
    with open(os.path.join(chart_dir, "Chart.yaml")) as f:
        chart_yaml = yaml.safe_load(f)
    chart = {"Name": chart_yaml["name"], "Version": chart_yaml["version"],
             "AppVersion": chart_yaml.get("appVersion", "")}
    r = Renderer(values, chart, {"Name": release, "Service": "Helm", "Namespace": values.get("namespace")})

    def get_file(path):  # .Files.Get: a file of the chart, "" if absent (as helm)
        try:
            with open(os.path.join(chart_dir, path)) as f:
                return f.read()
        except OSError:
            return ""
    r.root["Files"] = {"Get": get_file}
    tdir = os.path.join(chart_dir, "templates")
    parsed = {}
    for name in sorted(os.listdir(tdir)):
        with open(os.path.join(tdir, name)) as f:
            parsed[name] = r.load(f.read())
    for name, nodes in parsed.items():  # defines first (helpers)
        if name.startswith("_"):
            r.render_nodes(nodes, r.root, {})
    # NOTES.txt is what helm prints after an install, not a manifest (render_notes).
    return {name: r.render_nodes(nodes, r.root, {}) for name, nodes in parsed.items()
            if not name.startswith("_") and (notes or name != "NOTES.txt")}


def render_notes(values_override=None, release="amdgpu", chart_dir=CHART):
    """The text `helm install` prints (templates/NOTES.txt)."""
    return render(values_override, release, chart_dir, notes=True)["NOTES.txt"]


def _set(values, assignment):
    key, _, raw = assignment.partition("=")
    cur = values
    parts = key.split(".")
    for p in parts[:-1]:
        cur = cur.setdefault(p, {})
    cur[parts[-1]] = yaml.safe_load(raw)


if __name__ == "__main__":
    override = {}
    args = sys.argv[1:]
    while args:
        if args[0] == "--set" and len(args) > 1:
            _set(override, args[1])
            args = args[2:]
        else:
            raise SystemExit(__doc__)
    for name, text in render(override).items():
        sys.stdout.write(f"---\n# Source: {name}\n{text.strip()}\n")
