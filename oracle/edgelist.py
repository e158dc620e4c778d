"""CPU restatement of the edge-list ingest — TEST INFRASTRUCTURE ONLY (never
imported by the product path; the GPU parser is csrc/edge_list.hip).

Follows EdgeListDataSource.graph
(flink-cypher/src/main/scala/org/opencypher/flink/api/io/edgelist/EdgeListDataSource.scala:61-81):
a Flink CsvTableSource with two LONG fields, fieldDelimiter(options("sep")) and
commentPrefix(options("comment")) (:62-68), ids from safeAddIdColumn =
zipWithUniqueId (flink-cypher/.../impl/TableOps.scala:217-238), nodes =
distinct(source ∪ target) (:74-77).  Row rules restated from Flink 1.7's
CsvInputFormat.readRecord / GenericCsvInputFormat.parseRecord / LongParser
(third-party org.apache.flink:flink-java 1.7.0, not vendored): records split
at '\n', a trailing '\r' dropped, comment-prefixed records skipped, a LONG is
'-'? digits up to the delimiter, anything else (empty field, whitespace,
overflow, fewer than two fields) raises; bytes after the second field are
not read.  Parity pinned by the reference's EdgeListDataSourceTest
(morpheus-testing/.../api/io/edgelist/EdgeListDataSourceTest.scala:39-82:
4 nodes, 4 rels) and by hand-checked cases; Flink's own CSV behaviour on
malformed rows is "parity unpinned" (no JVM here).
"""
import numpy as np

INT64_MAX = (1 << 63) - 1


class ParseError(ValueError):
    def __init__(self, line, reason):
        super().__init__(f"edge list line {line} could not be parsed: {reason}")
        self.line = line
        self.reason = reason


def _parse_long(rec, p, sep):
    """LongParser over rec[p:] up to sep → (value, end index) or reason."""
    if p >= len(rec) or rec.startswith(sep, p):
        return None, "empty"
    neg = rec[p:p + 1] == b"-"
    if neg:
        p += 1
        if p >= len(rec) or rec.startswith(sep, p):
            return None, "orphan sign"
    limit = INT64_MAX + 1 if neg else INT64_MAX
    mag = 0
    while p < len(rec) and not rec.startswith(sep, p):
        c = rec[p]
        if not 48 <= c <= 57:
            return None, "illegal character"
        mag = mag * 10 + (c - 48)
        if mag > limit:
            return None, "overflow"
        p += 1
    return (-mag if neg else mag), p


def parse(data: bytes, sep: str, comment=None):
    """→ (ids, src, dst) int64 arrays; raises ParseError(line (1-based), reason)."""
    sepb = sep.encode()
    com = comment.encode() if comment else None
    if not sepb:
        raise ValueError("empty delimiter")
    recs = data.split(b"\n")
    if data.endswith(b"\n") or not data:
        recs = recs[:-1]  # the final delimiter ends the last record
    src, dst = [], []
    for i, rec in enumerate(recs):
        if rec.endswith(b"\r"):
            rec = rec[:-1]
        if com and rec.startswith(com):
            continue
        a, p = _parse_long(rec, 0, sepb)
        if a is None:
            raise ParseError(i + 1, p)
        if p >= len(rec):
            raise ParseError(i + 1, "row too short")
        p += len(sepb)
        if p >= len(rec):
            raise ParseError(i + 1, "row too short")
        b, q = _parse_long(rec, p, sepb)
        if b is None:
            raise ParseError(i + 1, q)
        src.append(a)
        dst.append(b)
    m = len(src)
    return (np.arange(m, dtype=np.int64), np.array(src, dtype=np.int64).reshape(m),
            np.array(dst, dtype=np.int64).reshape(m))


def nodes(src, dst):
    """distinct(source ∪ target) (EdgeListDataSource.scala:74-77), sorted."""
    return np.unique(np.concatenate([src, dst]))


def write_csv(src, dst, sep=",", crlf=False, comments=(), trailing_newline=True):
    """Bytes of an edge-list CSV; `comments` = [(line index, text)] inserted."""
    nl = "\r\n" if crlf else "\n"
    lines = [f"{a}{sep}{b}" for a, b in zip(src.tolist(), dst.tolist())]
    for idx, text in sorted(comments, reverse=True):
        lines.insert(idx, text)
    body = nl.join(lines)
    if trailing_newline and lines:
        body += nl
    return body.encode()
