"""FS graph source: property graphs stored as a directory of CSV tables.

Mirrors FSGraphSource over CsvFormat (flink-cypher/.../api/io/fs/FSGraphSource.scala:47-148,
GraphSources.fs(root).csv, api/GraphSources.scala:7-27) and the layout of
DefaultGraphDirectoryStructure (api/io/fs/GraphDirectoryStructure.scala:35-98):

    <root>/<graph name, '.' → '/'>/propertyGraphSchema.json   PropertyGraphSchema JSON
                                  /capsGraphMetaData.json      {"tableStorageFormat": "csv", "tags": [0]}
                                  /nodes/<labels sorted, '_'-joined, encoded>/<files>
                                  /relationships/<rel type, encoded>/<files>

Every table is read with the canonical field list of CAPFGraphExport
(api/io/util/CAPFGraphExport.scala: `id` for nodes, `id, source, target` for
relationships, then the properties sorted by their column name
`property_<encoded key>`), no header, ',' between fields, '\\n' between rows
— Flink's CsvTableSource defaults (FSGraphSource.scala:80-84).  A table
whose declared fields are all LONG (node/rel ids and INTEGER properties: the
shape of every R-MAT / LDBC edge table) is parsed on the GPU
(capf_csv_read_longs, csrc/edge_list.hip); tables with STRING / FLOAT /
BOOLEAN fields are parsed on the host and uploaded (strings are dictionary
codes, interned host-side).  `graph(name)` returns the ScanGraph of element
tables (AbstractPropertyGraphDataSource.graph, api/io/AbstractPropertyGraphDataSource.scala:87-108),
`store(name, graph)` writes one (:126-160).

Parity: the directory layout, schema JSON, column order and LONG row rules
are pinned by the reference's own CSV graph (flink-cypher/src/main/resources/
csv/products, committed as tests/golden/fs/products); how Flink's CSV source
treats an empty field, a BOOLEAN spelling or a DOUBLE format is not covered
by any reference fixture (parity unpinned): here an empty field is NULL,
BOOLEAN is true/false (any case), DOUBLE is Python float syntax.
"""
import json
import os
import shutil

from .expr import CT_TO_CAPF, T_BOOL, T_FLOAT, T_INT

SCHEMA_FILE = "propertyGraphSchema.json"
META_FILE = "capsGraphMetaData.json"
NODES_DIR = "nodes"
RELS_DIR = "relationships"
PROPERTY_PREFIX = "property_"


def encode_special(s):
    """StringEncodingUtilities.encodeSpecialCharacters (okapi-api/.../impl/util/
    StringEncodingUtilities.scala:73-95): ASCII letters, digits and '_' stay,
    every other char becomes '@' + 4 hex digits of each UTF-16 code unit."""
    out = []
    for ch in s:
        if ch == "_" or (ch.isascii() and ch.isalnum()):
            out.append(ch)
        else:
            b = ch.encode("utf-16-be")
            out.extend("@" + b[i:i + 2].hex() for i in range(0, len(b), 2))
    return "".join(out)


def decode_special(s):
    """decodeSpecialCharacters (:97-121)."""
    units, out, i = [], [], 0

    def flush():
        if units:
            out.append(b"".join(units).decode("utf-16-be"))
            units.clear()
    while i < len(s):
        if s[i] == "@":
            units.append(bytes.fromhex(s[i + 1:i + 5]))
            i += 5
        else:
            flush()
            out.append(s[i])
            i += 1
    flush()
    return "".join(out)


def node_table_dir(labels):
    """DefaultGraphDirectoryStructure.nodeTableDirectory (:66)."""
    return encode_special("_".join(sorted(labels)))


def _base_type(ct):
    """CypherType name of the schema JSON ('STRING', 'INTEGER?', …) → (base, nullable)."""
    return ct.rstrip("?"), ct.endswith("?")


def _canonical_props(props):
    """Properties in canonical column order: sorted by `property_<encoded key>`."""
    return sorted(props.items(), key=lambda kv: PROPERTY_PREFIX + encode_special(kv[0]))


class FSGraphSource:
    """A PropertyGraphDataSource over a directory tree of CSV tables."""

    def __init__(self, session, root, table_storage_format="csv"):
        if table_storage_format != "csv":
            raise NotImplementedError("only the CSV storage format is supported (ORC: no reader here)")
        self.session = session
        self.root = root
        self.table_storage_format = table_storage_format
        self._schema_cache = {}

    # -- DefaultGraphDirectoryStructure ------------------------------------------
    def graph_dir(self, name):
        return os.path.join(self.root, *name.split("."))

    def node_table_path(self, name, labels):
        return os.path.join(self.graph_dir(name), NODES_DIR, node_table_dir(labels))

    def rel_table_path(self, name, rel_type):
        return os.path.join(self.graph_dir(name), RELS_DIR, encode_special(rel_type))

    # -- catalog -----------------------------------------------------------------
    def graph_names(self):
        """listGraphNames = the directories under the root (FSGraphSource.scala:111-113)."""
        if not os.path.isdir(self.root):
            return set()
        return {d for d in os.listdir(self.root) if os.path.isdir(os.path.join(self.root, d))}

    def has_graph(self, name):
        return os.path.isfile(os.path.join(self.graph_dir(name), SCHEMA_FILE))

    def delete(self, name):
        self._schema_cache.pop(name, None)
        shutil.rmtree(self.graph_dir(name), ignore_errors=True)

    def schema(self, name):
        """PropertyGraphSchema.fromJson: {labels combo → {key: type}}, {rel type → {key: type}}."""
        if name not in self._schema_cache:
            with open(os.path.join(self.graph_dir(name), SCHEMA_FILE)) as f:
                js = json.load(f)
            if str(js.get("version", "1")).split(".")[0] != "1":
                raise ValueError("Incompatible Schema versions")
            nodes = {frozenset(e["labels"]): dict(e["properties"]) for e in js["labelPropertyMap"]}
            rels = {e["relType"]: dict(e["properties"]) for e in js["relTypePropertyMap"]}
            self._schema_cache[name] = (nodes, rels)
        return self._schema_cache[name]

    def metadata(self, name):
        with open(os.path.join(self.graph_dir(name), META_FILE)) as f:
            return json.load(f)

    # -- read ----------------------------------------------------------------------
    def graph(self, name, compact=False):
        """AbstractPropertyGraphDataSource.graph: one element table per label
        combination / relationship type of the schema."""
        from .graph import ElementTable, ScanGraph
        from .table import compact_as
        if not self.has_graph(name):
            raise KeyError(f"Graph with name '{name}' not found")
        nodes, rels = self.schema(name)
        node_tables, rel_tables = [], []
        for labels in sorted(nodes, key=lambda c: sorted(c)):
            props = nodes[labels]
            fields = [("id", "INTEGER")] + [(PROPERTY_PREFIX + encode_special(k), ct)
                                            for k, ct in _canonical_props(props)]
            t = self._read_table(self.node_table_path(name, labels), fields)
            t = t.select(*self._renames(fields))
            node_tables.append(ElementTable("node", labels, compact_as(t, compact),
                                            {k: _base_type(ct)[0] for k, ct in props.items()}))
        for rel_type in sorted(rels):
            props = rels[rel_type]
            fields = [("id", "INTEGER"), ("source", "INTEGER"), ("target", "INTEGER")] + \
                [(PROPERTY_PREFIX + encode_special(k), ct) for k, ct in _canonical_props(props)]
            t = self._read_table(self.rel_table_path(name, rel_type), fields)
            t = t.select(*self._renames(fields))
            rel_tables.append(ElementTable("rel", frozenset([rel_type]), compact_as(t, compact),
                                           {k: _base_type(ct)[0] for k, ct in props.items()}))
        return ScanGraph(self.session, node_tables, rel_tables)

    @staticmethod
    def _renames(fields):
        """Canonical CSV field names → the element-table columns of graph.py."""
        out = []
        for f, _ in fields:
            if f.startswith(PROPERTY_PREFIX):
                out.append((f, "p_" + decode_special(f[len(PROPERTY_PREFIX):])))
            else:
                out.append((f, f))
        return out

    def _files(self, path):
        if os.path.isfile(path):
            return [path]
        if not os.path.isdir(path):
            return []
        return [os.path.join(path, f) for f in sorted(os.listdir(path))
                if not f.startswith((".", "_")) and os.path.isfile(os.path.join(path, f))]

    def _read_table(self, path, fields):
        names = [f for f, _ in fields]
        types = [CT_TO_CAPF[_base_type(ct)[0]] for _, ct in fields]
        files = self._files(path)
        # The GPU LONG parser rejects an empty field; a nullable field ('INTEGER?')
        # stores NULL as an empty field, so such tables take the host reader.
        gpu = hasattr(self.session, "csv_read_longs") and not any(_base_type(ct)[1] for _, ct in fields)
        parts = []
        for fp in files:
            if gpu and all(t == T_INT for t in types):
                parts.append(self.session.csv_read_longs(fp, ",", names))
            else:
                parts.append(self.session.table(_parse_csv(fp, types, names)))
        if not parts:
            return self.session.empty(names, types)
        out = parts[0]
        for p in parts[1:]:
            out = out.unionAll(p)
        return out

    # -- write ---------------------------------------------------------------------
    def store(self, name, graph):
        """AbstractPropertyGraphDataSource.store: metadata, schema, then one CSV
        file per canonical node / relationship table."""
        if self.has_graph(name):
            raise ValueError(f"A graph with name {name} is already stored in this graph data source.")
        gdir = self.graph_dir(name)
        os.makedirs(gdir, exist_ok=True)
        with open(os.path.join(gdir, META_FILE), "w") as f:
            json.dump({"tableStorageFormat": self.table_storage_format, "tags": [0]}, f, indent=4)
        schema = {"version": "1.0",
                  "labelPropertyMap": [{"labels": sorted(t.labels), "properties": _schema_props(t)}
                                       for t in graph.node_tables],
                  "relTypePropertyMap": [{"relType": next(iter(t.labels)), "properties": _schema_props(t)}
                                         for t in graph.rel_tables]}
        with open(os.path.join(gdir, SCHEMA_FILE), "w") as f:
            json.dump(schema, f, indent=4)
        for t in graph.node_tables:
            cols = [t.id_col] + [t.prop_col(k) for k, _ in _canonical_props(t.props)]
            self._write_table(self.node_table_path(name, t.labels), t.table, cols)
        for t in graph.rel_tables:
            cols = [t.id_col, t.src_col, t.dst_col] + [t.prop_col(k) for k, _ in _canonical_props(t.props)]
            self._write_table(self.rel_table_path(name, next(iter(t.labels))), t.table, cols)
        self._schema_cache.pop(name, None)

    @staticmethod
    def _write_table(path, table, cols):
        os.makedirs(path, exist_ok=True)
        data = [table.column_values(c) for c in cols]
        with open(os.path.join(path, "part-00000.csv"), "w", newline="") as f:
            for row in zip(*data):
                f.write(",".join(_format_field(v) for v in row) + "\n")


def _schema_props(t):
    """Property types of an element table for the schema JSON: a property that
    is missing on some element (a NULL in its column) is nullable ('INTEGER?'),
    as okapi's PropertyGraphSchema types it — the reader then knows that an
    empty CSV field is NULL."""
    out = {}
    for k, ct in t.props.items():
        if not ct.endswith("?") and any(v is None for v in t.table.column_values(t.prop_col(k))):
            ct += "?"
        out[k] = ct
    return out


def _format_field(v):
    if v is None:
        return ""
    if isinstance(v, bool):
        return "true" if v else "false"
    return str(v)


def _parse_field(s, t, line, path):
    if s == "":
        return None
    try:
        if t == T_INT:
            if s.strip() != s or s.startswith("+"):
                raise ValueError(s)
            return int(s)
        if t == T_FLOAT:
            return float(s)
        if t == T_BOOL:
            low = s.lower()
            if low not in ("true", "false"):
                raise ValueError(s)
            return low == "true"
    except ValueError:
        raise ValueError(f"{path}: line {line} could not be parsed: {s!r} is not a {t}") from None
    return s


def _parse_csv(path, types, names):
    """Host CSV reader for tables with non-LONG fields: no quoting (Flink's
    CsvTableSource default), trailing '\\r' stripped, fields after the declared
    ones not read, a short row fails the read."""
    cols = [[] for _ in names]
    with open(path, encoding="utf-8") as f:
        for ln, line in enumerate(f, 1):
            line = line.rstrip("\n")
            if line.endswith("\r"):
                line = line[:-1]
            parts = line.split(",")
            if len(parts) < len(names):
                raise ValueError(f"{path}: line {ln} could not be parsed: Row too short")
            for i, t in enumerate(types):
                cols[i].append(_parse_field(parts[i], t, ln, path))
    return [(n, t, vals, None) for n, t, vals in zip(names, types, cols)]
