"""CREATE-string → in-memory property graph — TEST INFRASTRUCTURE ONLY.

Restates the id assignment of okapi-testing's CreateQueryParser
(okapi-testing/src/main/scala/org/opencypher/okapi/testing/propertygraph/
CreateQueryParser.scala:150-200, 302-309): nodes and relationships share ONE
id counter starting at 0, in processing order; a relationship chain is
processed left-nested — first element, then the target node, then the
relationship (so `(a)-[:R]->(b)-[:R]->(c)` assigns a=0, b=1, r1=2, c=3, r2=4);
variables that are already bound are reused; `<-[:T]-` stores the right node
as start.  Only the CREATE subset the reference's acceptance tests use is
supported (labels, property maps with ints/floats/strings/booleans/NULL).
"""
import re

from capf_amd.graph import GraphData

_TOKEN = re.compile(r"""
    (?P<ws>\s+)
  | (?P<kw>CREATE\b)
  | (?P<arrow_out>\]->)
  | (?P<arrow_in_start><-\[)
  | (?P<dash_open>-\[)
  | (?P<dash_close>\]-)
  | (?P<float>-?\d+\.\d*(?:[eE][-+]?\d+)?[dDfF]?|-?\d+[dD])
  | (?P<int>-?\d+)
  | (?P<str>'(?:[^'\\]|\\.)*'|"(?:[^"\\]|\\.)*")
  | (?P<name>[A-Za-z_][A-Za-z_0-9]*|`[^`]+`)
  | (?P<sym>[(){}:,\[\]])
""", re.VERBOSE)


def _tokens(s):
    pos = 0
    out = []
    while pos < len(s):
        m = _TOKEN.match(s, pos)
        if not m:
            raise ValueError(f"cannot tokenize at: {s[pos:pos + 20]!r}")
        pos = m.end()
        kind = m.lastgroup
        if kind == "ws":
            continue
        out.append((kind, m.group(kind)))
    return out


class _P:
    def __init__(self, toks):
        self.t = toks
        self.i = 0

    def peek(self, k=0):
        return self.t[self.i + k] if self.i + k < len(self.t) else (None, None)

    def take(self, kind=None, val=None):
        tok = self.peek()
        if kind and tok[0] != kind or val and tok[1] != val:
            raise ValueError(f"expected {kind} {val}, got {tok}")
        self.i += 1
        return tok

    def value(self):
        k, v = self.peek()
        if k == "int":
            self.i += 1
            return int(v)
        if k == "float":
            self.i += 1
            return float(v.rstrip("dDfF"))
        if k == "str":
            self.i += 1
            return bytes(v[1:-1], "utf-8").decode("unicode_escape")
        if k == "name" and v.upper() in ("NULL", "TRUE", "FALSE"):
            self.i += 1
            return {"NULL": None, "TRUE": True, "FALSE": False}[v.upper()]
        if k == "sym" and v == "[":  # a list property value (CTList)
            self.i += 1
            out = []
            while self.peek() != ("sym", "]"):
                out.append(self.value())
                if self.peek() == ("sym", ","):
                    self.take()
            self.take("sym", "]")
            return out
        raise ValueError(f"bad value {self.peek()}")

    def props(self):
        d = {}
        if self.peek() == ("sym", "{"):
            self.take("sym", "{")
            while self.peek() != ("sym", "}"):
                key = self.take("name")[1].strip("`")
                self.take("sym", ":")
                d[key] = self.value()
                if self.peek() == ("sym", ","):
                    self.take()
            self.take("sym", "}")
        return d


def parse_create(query):
    p = _P(_tokens(query))
    g = GraphData()
    nodes = {}          # var -> id
    counter = [0]

    def next_id():
        v = counter[0]
        counter[0] += 1
        return v

    anon = [0]

    def node():
        p.take("sym", "(")
        var = None
        if p.peek()[0] == "name":
            var = p.take()[1].strip("`")
        labels = []
        while p.peek() == ("sym", ":"):
            p.take()
            labels.append(p.take("name")[1].strip("`"))
        props = p.props()
        p.take("sym", ")")
        if var is not None and var in nodes:
            return nodes[var]
        nid = next_id()
        g.nodes.append((nid, frozenset(labels), props))
        if var is None:
            anon[0] += 1
            var = f"  anon{anon[0]}"
        nodes[var] = nid
        return nid

    def rel_head():
        incoming = p.peek()[0] == "arrow_in_start"
        p.take()
        if p.peek()[0] == "name":
            p.take()  # rel variable
        p.take("sym", ":")
        typ = p.take("name")[1].strip("`")
        props = p.props()
        closing = p.take()[0]
        if incoming and closing != "dash_close" or not incoming and closing != "arrow_out":
            raise ValueError("undirected or malformed relationship in CREATE")
        return typ, props, incoming

    def pattern():
        left = node()
        while p.peek()[0] in ("dash_open", "arrow_in_start"):
            typ, props, incoming = rel_head()
            right = node()
            rid = next_id()
            if incoming:
                g.rels.append((rid, right, left, typ, props))
            else:
                g.rels.append((rid, left, right, typ, props))
            left = right
        return left

    while p.peek()[0] is not None:
        p.take("kw")
        pattern()
        while p.peek() == ("sym", ","):
            p.take()
            pattern()
    return g
