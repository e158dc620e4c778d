"""Scanner for the JVM drop-in (integration/scala): which okapi classes,
extractors and inherited members the Scala sources use, and — given the
reference's Scala sources — what those names are there (kind, case-class
arity, declared members, parents).

Used by tests/golden/make_okapi_api.py (builds tests/golden/okapi_api.json
from /root/reference) and tests/test_scala_integration.py (checks the
integration sources against that fixture).  Regex level, not a Scala parser:
enough for the declaration forms the reference and the integration use.
"""
import os
import re

OKAPI = "org.opencypher.okapi"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCALA_DIR = os.path.join(ROOT, "integration", "scala", "org", "opencypher", "gpu")

_IMPORT = re.compile(r"^import\s+(org\.opencypher\.okapi[\w.]*?)\.(\{[^}]*\}|\w+|_)\s*$", re.M)
_DEF = re.compile(r"(?:^|\s)((?:case\s+class|case\s+object|class|trait|object|type|lazy\s+val|val|def))\s+(`?[\w$]+`?)")


def strip_comments(text):
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return re.sub(r"//[^\n]*", "", text)


def integration_sources():
    out = {}
    for f in sorted(os.listdir(SCALA_DIR)):
        if f.endswith(".scala"):
            with open(os.path.join(SCALA_DIR, f)) as fh:
                out[f] = fh.read()
    return out


def imports(text):
    """[(prefix, name)] of okapi imports; name '_' for a wildcard."""
    out = []
    for m in _IMPORT.finditer(strip_comments(text)):
        prefix, sel = m.group(1), m.group(2)
        if sel.startswith("{"):
            for part in sel[1:-1].split(","):
                name = part.split("=>")[0].strip()
                if name:
                    out.append((prefix, name))
        else:
            out.append((prefix, sel))
    return out


def patterns(text):
    """Extractor patterns `case Name(args)` (name, arity) and bare `case Name =>`."""
    body = strip_comments(text)
    calls, bare = [], []
    for m in re.finditer(r"\bcase\s+([A-Z]\w*)\s*\(", body):
        if body[m.start():m.start() + 10].startswith("case class"):
            continue
        args = _balanced(body, m.end() - 1)
        calls.append((m.group(1), _arity(args)))
    for m in re.finditer(r"\bcase\s+([A-Z]\w*)\s*(?:=>|\|)", body):
        bare.append(m.group(1))
    return calls, bare


def classes(text):
    """{class name: (parent simple names, overridden member names)} of the
    classes / traits defined in a Scala source."""
    body = strip_comments(text)
    out = {}
    for m in re.finditer(r"\b(?:case\s+class|class|trait|object)\s+(\w+)", body):
        name = m.group(1)
        head_end = body.find("{", m.end())
        nxt = re.search(r"\n(?:case\s+class|final\s+class|class|trait|object|sealed|abstract)\b", body[m.end():])
        stop = m.end() + nxt.start() if nxt else len(body)
        if head_end < 0 or head_end > stop:
            head, block = body[m.end():stop], ""
        else:
            head = body[m.end():head_end]
            block = _balanced(body, head_end, "{", "}")
        head = _drop_parens(head)
        parents = re.findall(r"(?:extends|with)\s+([A-Z]\w*)", head)
        over = re.findall(r"\boverride\s+(?:protected\s+|private\[\w+\]\s+)?(?:lazy\s+val|val|def|type)\s+(\w+)", block)
        over += re.findall(r"\boverride\s+val\s+(\w+)\s*:", head)
        prev = out.get(name, ([], []))  # a class and its companion object merge
        out[name] = (prev[0] + parents, prev[1] + over)
    return out


def _drop_parens(s):
    out, depth = [], 0
    for ch in s:
        if ch in "([":
            depth += 1
        elif ch in ")]":
            depth -= 1
        elif depth == 0:
            out.append(ch)
    return "".join(out)


def _balanced(text, i, o="(", c=")"):
    """The text inside the bracket pair opening at text[i]."""
    depth = 0
    for j in range(i, len(text)):
        if text[j] == o:
            depth += 1
        elif text[j] == c:
            depth -= 1
            if depth == 0:
                return text[i + 1:j]
    return text[i + 1:]


def _arity(args):
    """Number of top-level comma-separated items of a parameter / argument list."""
    args = args.strip()
    if not args:
        return 0
    depth, n = 0, 1
    for ch in args:
        if ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
        elif ch == "," and depth == 0:
            n += 1
    return n


# ------------------------------------------------------------ reference side
def reference_files(ref_root):
    out = []
    for d, _, fs in os.walk(ref_root):
        if "/src/main/scala" not in d:
            continue
        for f in fs:
            if f.endswith(".scala"):
                out.append(os.path.join(d, f))
    return sorted(out)


def _package_of(text):
    m = re.search(r"^package\s+([\w.]+)", text, re.M)
    return m.group(1) if m else ""


def index_reference(ref_root):
    """{package: [(path, text)]} of the reference's main Scala sources."""
    idx = {}
    for p in reference_files(ref_root):
        with open(p, encoding="utf-8", errors="replace") as f:
            t = strip_comments(f.read())
        idx.setdefault(_package_of(t), []).append((p, t))
    return idx


def _definitions(text, name):
    """(kind, first-parameter-list arity or None) of every definition of `name`."""
    out = []
    for m in re.finditer(r"(?:^|[\s(])((?:case\s+class|case\s+object|class|trait|object|type|lazy\s+val|val|def))\s+"
                         + re.escape(name) + r"\b", text):
        kind = re.sub(r"\s+", " ", m.group(1))
        arity = None
        if kind == "case class":
            rest = text[m.end():]
            k = 0
            while k < len(rest) and rest[k] in " \t":
                k += 1
            if rest[k:k + 1] == "[":
                k += len(_balanced(rest, k, "[", "]")) + 2
            if rest[k:k + 1] == "(":
                arity = _arity(_balanced(rest, k))
        elif kind == "object":
            # an extractor object: UnapplyValue (one value) or its own unapply
            head_end = text.find("{", m.end())
            nl = text.find("\n", m.end())
            head = text[m.end():nl if 0 <= nl < head_end or head_end < 0 else head_end]
            if re.search(r"extends\s+UnapplyValue\b", head):
                arity = 1
            elif head_end >= 0 and (nl < 0 or head_end <= nl):
                body = _balanced(text, head_end, "{", "}")
                u = re.search(r"def\s+unapply\b[^:]*\)\s*:\s*Option\[", body)
                if u:
                    inner = _balanced(body, u.end() - 1, "[", "]").strip()
                    arity = _arity(_balanced(inner, 0)) if inner.startswith("(") else 1
        out.append((kind, arity))
    return out


def resolve(idx, prefix, name):
    """Definitions of prefix.name in the reference: prefix is a package, or a
    package plus an object path (org.opencypher.okapi.api.value.CypherValue)."""
    parts = prefix.split(".")
    for cut in range(len(parts), 0, -1):
        pkg, objs = ".".join(parts[:cut]), parts[cut:]
        files = idx.get(pkg)
        if not files:
            continue
        found = []
        for _, t in files:
            scope = t
            ok = True
            for o in objs:
                m = re.search(r"\bobject\s+" + re.escape(o) + r"\b[^{]*\{", t)
                if not m:
                    ok = False
                    break
                scope = _balanced(t, m.end() - 1, "{", "}")
            if ok:
                found += _definitions(scope, name)
        if found:
            return found
    return []


def package_names(idx, pkg):
    """Names defined in a package, or in an object (package + object path),
    that a wildcard import brings in."""
    names = set()
    decl = r"(?:final\s+|sealed\s+|abstract\s+|implicit\s+)*(?:case\s+class|case\s+object|class|trait|object)\s+(\w+)"
    if pkg in idx:
        for _, t in idx[pkg]:
            names.update(m.group(1) for m in re.finditer(r"^" + decl, t, re.M))
        return names
    prefix, obj = pkg.rsplit(".", 1)
    for _, t in idx.get(prefix, []):
        m = re.search(r"\bobject\s+" + re.escape(obj) + r"\b[^{]*\{", t)
        if m:
            names.update(x.group(1) for x in re.finditer(decl, _balanced(t, m.end() - 1, "{", "}")))
    return names


def _type_decl(text, name):
    return re.search(r"(?:^|\s)(?:trait|abstract\s+class|class)\s+" + re.escape(name) + r"\b", text)


def members_of(idx, name, prefix=None, near=None):
    """Declared member names and parent names of trait / class `name`, and
    where it was found: looked up in `prefix` (a package or package.object
    path) first, then next to `near` (the child's (package, file text)), then
    anywhere in the reference's main sources."""
    scopes = []
    if prefix:
        parts = prefix.split(".")
        for cut in range(len(parts), 0, -1):
            pkg, objs = ".".join(parts[:cut]), parts[cut:]
            for _, t in idx.get(pkg, []):
                scope = t
                for o in objs:
                    m = re.search(r"\bobject\s+" + re.escape(o) + r"\b[^{]*\{", scope)
                    scope = _balanced(scope, m.end() - 1, "{", "}") if m else None
                    if scope is None:
                        break
                if scope is not None:
                    scopes.append((pkg, scope))
            if scopes:
                break
    if near:
        scopes.append(near)
        scopes += [(near[0], t) for _, t in idx.get(near[0], [])]
    scopes += [(pkg, t) for pkg, files in idx.items() for _, t in files]
    for pkg, t in scopes:
        m = _type_decl(t, name)
        if not m:
            continue
        brace = t.find("{", m.end())
        nxt = re.search(r"\n\s*(?:final\s+|sealed\s+|abstract\s+)*(?:case\s+class|class|trait|object)\b", t[m.end():])
        if brace < 0 or (nxt and m.end() + nxt.start() < brace):
            head, block = t[m.end():m.end() + (nxt.start() if nxt else 200)], ""
        else:
            head, block = t[m.end():brace], _balanced(t, brace, "{", "}")
        parents = re.findall(r"(?:extends|with)\s+([A-Z]\w*)", _drop_parens(head))
        depth, members = 0, set()
        for line in block.split("\n"):
            if depth == 0:
                mm = re.search(r"\b(?:lazy\s+val|val|def|type)\s+(\w+)", line)
                if mm:
                    members.add(mm.group(1))
            depth += line.count("{") - line.count("}")
        return sorted(members), parents, (pkg, t)
    return None
