"""Golden cases transcribed from the reference's own acceptance tests.

Each case = (id, reference file:line, CREATE graph, query, expected Bag).  The
CREATE strings and expected bags are copied verbatim (as data) from the
reference tests; the query is the Cypher query expressed in the planner's
pattern model (the Cypher parser / IR builder are out of scope).

Sources (relative to the reference checkout):
  FTm = flink-cypher-testing/src/main/scala/org/opencypher/flink/test/
  FTt = flink-cypher-testing/src/test/scala/org/apache/flink/impl/
  MTa = morpheus-testing/src/test/scala/org/opencypher/morpheus/impl/acceptance/
"""
import capf_import  # noqa: F401
from capf_amd.expr import (Avg, Collect, Count, CountStar, ElementProperty, Exists, FloatLit, Id, In, IntegerLit, ListLit,
                           Max, Min, NullLit, Param, Size, StringLit, Sum, Type, Var)
from capf_amd.planner import Match, NodeP, Query, RelP, Stage


def P(v, k, ct="ANY"):
    return ElementProperty(Var(v, "NODE"), k, ct)


def N(v):
    return Var(v, "NODE")


TEAM = """
       CREATE (a:Person:German {name: "Stefan", luckyNumber: 42})
       CREATE (b:Person:Swede  {name: "Mats", luckyNumber: 23})
       CREATE (c:Person:German {name: "Martin", luckyNumber: 1337})
       CREATE (d:Person:German {name: "Max", luckyNumber: 8})
       CREATE (a)-[:KNOWS {since: 2016}]->(b)
       CREATE (b)-[:KNOWS {since: 2016}]->(c)
       CREATE (c)-[:KNOWS {since: 2016}]->(d)
"""

SIX = "CREATE ({name: 'foo'}), ({name: 'bar'}), (), (), (), ({name: 'baz'})"
INTS = "CREATE ({val: 2}),({val: 4}),({val: 6})"
FLOATS = "CREATE ({val:5.0D}),({val:5.0D}),({val:0.5D})"
FLOATS_NULL = "CREATE ({val:42.0D}),({val:23.0D}),()"
NULLS = "CREATE ({val:NULL}),(),()"
INTS3 = "CREATE ({val: 42}),({val: 23}),({val: 84})"
INTS_NULL = "CREATE ({val: 42}),({val: 23}),()"


def ret(*items, **kw):
    return Stage(list(items), **kw)


def scan_n(*stages):
    return Query([Match([NodeP("n")])], list(stages))


CASES = [
    # ---------------------------------------------------------------- config 1
    ("team_knows", "FTm/fixture/TeamDataFixture.scala:47-56 (SURVEY §8(c)1)", TEAM,
     Query([Match([NodeP("a", ("Person",)), NodeP("b")], [RelP("r", "a", "b", ("KNOWS",))])],
           [ret(("a.name", P("a", "name")), ("b.name", P("b", "name")))]),
     [{"a.name": "Stefan", "b.name": "Mats"}, {"a.name": "Mats", "b.name": "Martin"},
      {"a.name": "Martin", "b.name": "Max"}]),

    # ---------------------------------------------------- BoundedVarExpandTests
    ("varlen_zero_length", "FTt/acceptance/BoundedVarExpandTests.scala:38-58",
     "CREATE (n0:A {name: 'n0'}), (n00:B {name: 'n00'}) CREATE (n0)-[:LIKES]->(n00)",
     Query([Match([NodeP("a", ("A",))]),
            Match([NodeP("a"), NodeP("c")], [RelP("r", "a", "c", ("LIKES",), length=(0, 0))])],
           [ret(("c.name", P("c", "name")))]),
     [{"c.name": "n0"}]),
    ("varlen_0_1", "FTt/acceptance/BoundedVarExpandTests.scala:60-79",
     "CREATE (s:Node {val: 'source'})-[:REL]->(:Node {val: 'mid1'})-[:REL]->(:Node {val: 'end'})",
     Query([Match([NodeP("n", ("Node",)), NodeP("m", ("Node",))], [RelP("r", "n", "m", length=(0, 1))])],
           [ret(("m.val", P("m", "val")))]),
     [{"m.val": "source"}, {"m.val": "mid1"}, {"m.val": "mid1"}, {"m.val": "end"}, {"m.val": "end"}]),
    ("varlen_lower_bound", "FTt/acceptance/BoundedVarExpandTests.scala:81-95",
     "CREATE (:Node {val: 'source'})-[:REL]->(:Node {val: 'mid1'})-[:REL]->(:Node {val: 'end'})",
     Query([Match([NodeP("t", ("Node",)), NodeP("y", ("Node",))], [RelP("r", "t", "y", length=(2, 3))])],
           [ret(("y.val", P("y", "val")))]),
     [{"y.val": "end"}]),
    ("varlen_loop", "FTt/acceptance/BoundedVarExpandTests.scala:97-118",
     "CREATE (a:Node {v: 'a'})-[:REL]->(:Node {v: 'b'})-[:REL]->(:Node {v: 'c'})-[:REL]->(a)",
     Query([Match([NodeP("a", ("Node",)), NodeP("b", ("Node",))], [RelP("r", "a", "b", length=(1, 6))])],
           [ret(("b.v", P("b", "v")))]),
     [{"b.v": "a"}] * 3 + [{"b.v": "b"}] * 3 + [{"b.v": "c"}] * 3),
    ("varlen_rel_type", "FTt/acceptance/BoundedVarExpandTests.scala:145-158",
     "CREATE (a:Node {v: 'a'})-[:LOVES]->(:Node {v: 'b'})-[:KNOWS]->(:Node {v: 'c'})-[:HATES]->(a)",
     Query([Match([NodeP("a", ("Node",)), NodeP("b", ("Node",))],
                  [RelP("r", "a", "b", ("LOVES", "KNOWS"), length=(1, 6))])],
           [ret(("b.v", P("b", "v")))]),
     [{"b.v": "b"}, {"b.v": "c"}, {"b.v": "c"}]),
    ("varlen_additional_hop", "FTt/acceptance/BoundedVarExpandTests.scala:178-190",
     "CREATE (a:Node {v: 'a'})-[:KNOWS]->(:Node {v: 'b'})-[:KNOWS]->(:Node {v: 'c'})-[:HATES]->(d:Node {v: 'd'})",
     Query([Match([NodeP("a", ("Node",)), NodeP("b", ("Node",)), NodeP("c", ("Node",))],
                  [RelP("r", "a", "b", ("KNOWS",), length=(1, 6)), RelP("h", "b", "c", ("HATES",))])],
           [ret(("c.v", P("c", "v")))]),
     [{"c.v": "d"}, {"c.v": "d"}]),
    ("varlen_expand_into", "FTt/acceptance/BoundedVarExpandTests.scala:192-215",
     """CREATE (a:Person {name: "Philip"})
        CREATE (b:Person {name: "Stefan"})
        CREATE (c:City {name: "Berlondon"})
        CREATE (a)-[:KNOWS]->(b)
        CREATE (a)-[:LIVES_IN]->(c)
        CREATE (b)-[:LIVES_IN]->(c)""",
     Query([Match([NodeP("a", ("Person",)), NodeP("c", ("City",)), NodeP("b", ("Person",))],
                  [RelP("l1", "a", "c", ("LIVES_IN",)), RelP("l2", "b", "c", ("LIVES_IN",)),
                   RelP("k", "a", "b", ("KNOWS",), length=(1, 2))])],
           [ret(("a.name", P("a", "name")), ("b.name", P("b", "name")), ("c.name", P("c", "name")))]),
     [{"a.name": "Philip", "b.name": "Stefan", "c.name": "Berlondon"}]),

    # ---------------------------------------------------------- AggregationTests
    # avg over INTEGER values is a FLOAT (4.0): the reference test's expected
    # CypherMap("res" -> 4) equals it only under Scala Map equality, whose
    # numeric comparison is cooperative (CypherValue.scala:199-203, 301-302) —
    # option "coop"; every other case compares typed
    ("avg_ints", "FTt/acceptance/AggregationTests.scala:49-57", INTS,
     scan_n(ret(("res", Avg(P("n", "val"))))), [{"res": 4}], {"coop": True}),
    ("avg_floats", "FTt/acceptance/AggregationTests.scala:79-87", FLOATS,
     scan_n(ret(("res", Avg(P("n", "val"))))), [{"res": 3.5}]),
    ("avg_single_null", "FTt/acceptance/AggregationTests.scala:99-107", FLOATS_NULL,
     scan_n(ret(("res", Avg(P("n", "val"))))), [{"res": 32.5}]),
    ("avg_only_nulls", "FTt/acceptance/AggregationTests.scala:119-127", NULLS,
     scan_n(ret(("res", Avg(P("n", "val"))))), [{"res": None}]),
    ("count_star", "FTt/acceptance/AggregationTests.scala:150-158", SIX,
     scan_n(ret(("nbrRows", CountStar()))), [{"nbrRows": 6}]),
    ("count_n", "FTt/acceptance/AggregationTests.scala:160-168", SIX,
     scan_n(ret(("nbrRows", Count(N("n"))))), [{"nbrRows": 6}]),
    ("count_prop", "FTt/acceptance/AggregationTests.scala:190-198", SIX,
     scan_n(ret(("nonNullNames", Count(P("n", "name"))))), [{"nonNullNames": 3}]),
    ("count_after_expand", "FTt/acceptance/AggregationTests.scala:210-218",
     "CREATE ({name: 'foo'})-[:A]->(:B), ({name: 'bar'}), (), ()-[:A]->(:B), (), ({name: 'baz'})",
     Query([Match([NodeP("n"), NodeP("b", ("B",))], [RelP("r", "n", "b")])],
           [ret(("nodes", Count(N("b"))))]),
     [{"nodes": 2}]),
    ("count_grouping", "FTt/acceptance/AggregationTests.scala:220-230",
     "CREATE ({name: 'foo'}), ({name: 'foo'}), (), (), (), ({name: 'baz'})",
     scan_n(ret(("name", P("n", "name")), ("amount", CountStar()))),
     [{"name": "foo", "amount": 2}, {"name": None, "amount": 3}, {"name": "baz", "amount": 1}]),
    ("count_grouping_multi", "FTt/acceptance/AggregationTests.scala:244-256",
     "CREATE ({name: 'foo', age: 42}), ({name: 'foo', age: 42}), ({name: 'foo', age: 23}), (), (), "
     "({name: 'baz', age: 23})",
     scan_n(ret(("name", P("n", "name")), ("age", P("n", "age")), ("amount", CountStar()))),
     [{"name": "foo", "age": 23, "amount": 1}, {"name": "foo", "age": 42, "amount": 2},
      {"name": "baz", "age": 23, "amount": 1}, {"name": None, "age": None, "amount": 2}]),
    ("min_ints", "FTt/acceptance/AggregationTests.scala:292-300", INTS3,
     scan_n(ret(("res", Min(P("n", "val"))))), [{"res": 23}]),
    ("min_single_null", "FTt/acceptance/AggregationTests.scala:312-320", INTS_NULL,
     scan_n(ret(("res", Min(P("n", "val"))))), [{"res": 23}]),
    ("min_only_nulls", "FTt/acceptance/AggregationTests.scala:342-350", NULLS,
     scan_n(ret(("res", Min(P("n", "val"))))), [{"res": None}]),
    ("max_ints", "FTt/acceptance/AggregationTests.scala:397-405", INTS3,
     scan_n(ret(("res", Max(P("n", "val"))))), [{"res": 84}]),
    ("max_single_null", "FTt/acceptance/AggregationTests.scala:417-425", INTS_NULL,
     scan_n(ret(("res", Max(P("n", "val"))))), [{"res": 42}]),
    ("max_only_nulls", "FTt/acceptance/AggregationTests.scala:447-455", NULLS,
     scan_n(ret(("res", Max(P("n", "val"))))), [{"res": None}]),
    ("sum_ints", "FTt/acceptance/AggregationTests.scala:504-512", INTS,
     scan_n(ret(("res", Sum(P("n", "val"))))), [{"res": 12}]),
    ("sum_floats", "FTt/acceptance/AggregationTests.scala:524-532", FLOATS,
     scan_n(ret(("res", Sum(P("n", "val"))))), [{"res": 10.5}]),
    ("sum_single_null", "FTt/acceptance/AggregationTests.scala:554-562", FLOATS_NULL,
     scan_n(ret(("res", Sum(P("n", "val"))))), [{"res": 65.0}]),
    ("sum_only_nulls", "FTt/acceptance/AggregationTests.scala:574-582", NULLS,
     scan_n(ret(("res", Sum(P("n", "val"))))), [{"res": None}]),

    # ------------------------------------- shared okapi planner, Spark backend
    ("cyphermorphism_multi_match", "MTa/MatchTests.scala:142-177",
     """CREATE (p1:Person {name: "Alice"})
        CREATE (p2:Person {name: "Bob"})
        CREATE (p1)-[:KNOWS]->(p2)
        CREATE (p2)-[:KNOWS]->(p1)""",
     Query([Match([NodeP("p1", ("Person",)), NodeP("p2", ("Person",)), NodeP("p3", ("Person",))],
                  [RelP("e1", "p1", "p2", ("KNOWS",)), RelP("e2", "p2", "p3", ("KNOWS",))]),
            Match([NodeP("p3"), NodeP("p4", ("Person",))], [RelP("e3", "p3", "p4", ("KNOWS",))])],
           [ret(("p1.name", P("p1", "name")), ("p2.name", P("p2", "name")), ("p3.name", P("p3", "name")),
                ("p4.name", P("p4", "name")))]),
     [{"p1.name": "Bob", "p2.name": "Alice", "p3.name": "Bob", "p4.name": "Alice"},
      {"p1.name": "Alice", "p2.name": "Bob", "p3.name": "Alice", "p4.name": "Bob"}]),
    ("undirected_two_hops", "MTa/MatchTests.scala:273-294",
     """CREATE (a:A {prop: 'a'})
        CREATE (b:B {prop: 'b'})
        CREATE (c:C {prop: 'c'})
        CREATE (d:D {prop: 'd'})
        CREATE (a)-[:T]->(b)
        CREATE (b)-[:T]->(c)
        CREATE (c)-[:T]->(a)
        CREATE (c)-[:T]->(d)""",
     Query([Match([NodeP("a", ("A",)), NodeP("x"), NodeP("other")],
                  [RelP("r1", "a", "x", direction="both"), RelP("r2", "x", "other", direction="both")])],
           [ret(("a.prop", P("a", "prop")), ("other.prop", P("other", "prop")))]),
     [{"a.prop": "a", "other.prop": "c"}, {"a.prop": "a", "other.prop": "b"},
      {"a.prop": "a", "other.prop": "d"}]),
    ("mixed_directed_undirected", "MTa/MatchTests.scala:318-341",
     """CREATE (a:A {prop: 'a'})
        CREATE (b:B {prop: 'b'})
        CREATE (c:C {prop: 'c'})
        CREATE (a)-[:T]->(a)
        CREATE (a)-[:T]->(a)
        CREATE (b)-[:T]->(a)
        CREATE (a)-[:T]->(c)""",
     Query([Match([NodeP("a", ("A",)), NodeP("other")],
                  [RelP("r1", "a", "a", direction="both"), RelP("r2", "other", "a")])],
           [ret(("a.prop", P("a", "prop")), ("other.prop", P("other", "prop")))]),
     [{"a.prop": "a", "other.prop": "a"}, {"a.prop": "a", "other.prop": "a"},
      {"a.prop": "a", "other.prop": "b"}, {"a.prop": "a", "other.prop": "b"}]),
    ("undirected_cyclic", "MTa/MatchTests.scala:343-358",
     """CREATE (a:A {prop: 'isA'})
        CREATE (b:B)
        CREATE (a)-[:T]->(a)
        CREATE (b)-[:T]->(a)""",
     Query([Match([NodeP("a", ("A",))], [RelP("r", "a", "a", direction="both")])],
           [ret(("a.prop", P("a", "prop")))]),
     [{"a.prop": "isA"}]),
    ("expand_into_dangling", "MTa/ExpandIntoTests.scala:35-77",
     """CREATE (p1:Person {name: "Alice"})
        CREATE (p2:Person {name: "Bob"})
        CREATE (p3:Person {name: "Eve"})
        CREATE (p4:Person {name: "Carl"})
        CREATE (p5:Person {name: "Richard"})
        CREATE (p1)-[:KNOWS]->(p2)
        CREATE (p2)-[:KNOWS]->(p3)
        CREATE (p1)-[:KNOWS]->(p3)
        CREATE (p3)-[:KNOWS]->(p4)
        CREATE (p3)-[:KNOWS]->(p5)""",
     Query([Match([NodeP("p1", ("Person",)), NodeP("p2", ("Person",)), NodeP("p3", ("Person",)), NodeP("p4")],
                  [RelP("e1", "p1", "p2", ("KNOWS",)), RelP("e2", "p2", "p3", ("KNOWS",)),
                   RelP("e3", "p1", "p3", ("KNOWS",)), RelP("e4", "p3", "p4", ("KNOWS",))])],
           [ret(("p1.name", P("p1", "name")), ("p2.name", P("p2", "name")), ("p3.name", P("p3", "name")),
                ("p4.name", P("p4", "name")))]),
     [{"p1.name": "Alice", "p2.name": "Bob", "p3.name": "Eve", "p4.name": "Carl"},
      {"p1.name": "Alice", "p2.name": "Bob", "p3.name": "Eve", "p4.name": "Richard"}]),
    ("expand_into_triangle", "MTa/ExpandIntoTests.scala:78-107",
     """CREATE (p1:Person {name: "Alice"})
        CREATE (p2:Person {name: "Bob"})
        CREATE (p3:Person {name: "Eve"})
        CREATE (p1)-[:KNOWS]->(p2)
        CREATE (p2)-[:KNOWS]->(p3)
        CREATE (p1)-[:KNOWS]->(p3)""",
     Query([Match([NodeP("p1", ("Person",)), NodeP("p2", ("Person",)), NodeP("p3", ("Person",))],
                  [RelP("e1", "p1", "p2", ("KNOWS",)), RelP("e2", "p2", "p3", ("KNOWS",)),
                   RelP("e3", "p1", "p3", ("KNOWS",))])],
           [ret(("p1.name", P("p1", "name")), ("p2.name", P("p2", "name")), ("p3.name", P("p3", "name")))]),
     [{"p1.name": "Alice", "p2.name": "Bob", "p3.name": "Eve"}]),
]

CASES.append(
    ("undirected_var_length", "MTa/MatchTests.scala:360-376",
     """CREATE (a:A {prop: 'a'})
        CREATE (b:B {prop: 'b'})
        CREATE (c:C {prop: 'c'})
        CREATE (a)-[:T]->(b)
        CREATE (b)<-[:T]-(c)""",
     Query([Match([NodeP("a", ("A",)), NodeP("other")], [RelP("r", "a", "other", direction="both", length=(2, 2))])],
           [ret(("a.prop", P("a", "prop")), ("other.prop", P("other", "prop")))]),
     [{"a.prop": "a", "other.prop": "c"}]))


# ------------------------------------------------------ OptionalMatchTests (MTa)
# OPTIONAL MATCH = planOptional's left outer join (RelationalPlanner.scala:298-329),
# shared with the Flink backend through the okapi planner.
KNOWS3 = """
        CREATE (p1:Person {name: "Alice"})
        CREATE (p2:Person {name: "Bob"})
        CREATE (p3:Person {name: "Eve"})
        CREATE (p1)-[:KNOWS]->(p2)
        CREATE (p2)-[:KNOWS]->(p3)
"""


def _names(*vs):
    return ret(*[(f"{v}.name", P(v, "name")) for v in vs])


OPTIONAL_CASES = [
    ("optional_match", "MTa/OptionalMatchTests.scala:122-159", KNOWS3,
     Query([Match([NodeP("p1", ("Person",))]),
            Match([NodeP("p1"), NodeP("p2"), NodeP("p3")], [RelP("e1", "p1", "p2"), RelP("e2", "p2", "p3")],
                  optional=True)], [_names("p1", "p2", "p3")]),
     [{"p1.name": "Eve", "p2.name": None, "p3.name": None},
      {"p1.name": "Bob", "p2.name": None, "p3.name": None},
      {"p1.name": "Alice", "p2.name": "Bob", "p3.name": "Eve"}]),
    ("optional_match_predicates", "MTa/OptionalMatchTests.scala:161-189",
     """CREATE (p1:Person {name: "Alice"})
        CREATE (p2:Person {name: "Bob"})
        CREATE (p1)-[:KNOWS]->(p2)""",
     Query([Match([NodeP("p1", ("Person",))]),
            Match([NodeP("p1"), NodeP("p2", ("Person",))], [RelP("e1", "p1", "p2", ("KNOWS",))],
                  optional=True)], [_names("p1", "p2")]),
     [{"p1.name": "Bob", "p2.name": None}, {"p1.name": "Alice", "p2.name": "Bob"}]),
    ("optional_match_matched_rels", "MTa/OptionalMatchTests.scala:191-239",
     KNOWS3 + "        CREATE (p1)-[:KNOWS]->(p3)\n",
     Query([Match([NodeP("p1", ("Person",)), NodeP("p2", ("Person",))], [RelP("e1", "p1", "p2", ("KNOWS",))]),
            Match([NodeP("p1"), NodeP("p3", ("Person",))], [RelP("e2", "p1", "p3", ("KNOWS",))],
                  optional=True)], [_names("p1", "p2", "p3")]),
     [{"p1.name": "Alice", "p2.name": "Bob", "p3.name": "Eve"},
      {"p1.name": "Alice", "p2.name": "Eve", "p3.name": "Bob"},
      {"p1.name": "Alice", "p2.name": "Bob", "p3.name": "Bob"},
      {"p1.name": "Alice", "p2.name": "Eve", "p3.name": "Eve"},
      {"p1.name": "Bob", "p2.name": "Eve", "p3.name": "Eve"}]),
    ("optional_match_partial", "MTa/OptionalMatchTests.scala:276-313", KNOWS3,
     Query([Match([NodeP("p1", ("Person",))]),
            Match([NodeP("p1"), NodeP("p2", ("Person",)), NodeP("p3", ("Person",))],
                  [RelP("e1", "p1", "p2", ("KNOWS",)), RelP("e2", "p2", "p3", ("KNOWS",))], optional=True)],
           [_names("p1", "p2", "p3")]),
     [{"p1.name": "Alice", "p2.name": "Bob", "p3.name": "Eve"},
      {"p1.name": "Bob", "p2.name": None, "p3.name": None},
      {"p1.name": "Eve", "p2.name": None, "p3.name": None}]),
    ("optional_match_duplicates", "MTa/OptionalMatchTests.scala:315-351",
     """CREATE (p1:Person {name: "Alice"})
        CREATE (p2:Person {name: "Bob"})
        CREATE (p3:Person {name: "Eve"})
        CREATE (p4:Person {name: "Paul"})
        CREATE (p1)-[:KNOWS]->(p3)
        CREATE (p2)-[:KNOWS]->(p3)
        CREATE (p3)-[:KNOWS]->(p4)""",
     Query([Match([NodeP("a", ("Person",)), NodeP("b", ("Person",))], [RelP("e1", "a", "b", ("KNOWS",))]),
            Match([NodeP("b"), NodeP("c", ("Person",))], [RelP("e2", "b", "c", ("KNOWS",))], optional=True)],
           [_names("b", "c")]),
     [{"b.name": "Eve", "c.name": "Paul"}, {"b.name": "Eve", "c.name": "Paul"},
      {"b.name": "Paul", "c.name": None}]),
]
OPTIONAL_CASES.append(
    ("optional_match_duplicates_cycle", "MTa/OptionalMatchTests.scala:353-402",
     """CREATE (p1:Person {name: "Alice"})
        CREATE (p2:Person {name: "Bob"})
        CREATE (p3:Person {name: "Eve"})
        CREATE (p4:Person {name: "Paul"})
        CREATE (p1)-[:KNOWS]->(p3)
        CREATE (p2)-[:KNOWS]->(p3)
        CREATE (p3)-[:KNOWS]->(p4)
        CREATE (p4)-[:KNOWS {foo: 42}]->(p1)""",
     Query([Match([NodeP("a", ("Person",)), NodeP("b", ("Person",)), NodeP("c", ("Person",))],
                  [RelP("e1", "a", "b", ("KNOWS",)), RelP("e2", "b", "c", ("KNOWS",))]),
            Match([NodeP("c"), NodeP("a")], [RelP("e3", "c", "a", ("KNOWS",))], optional=True)],
           [ret(("a.name", P("a", "name")), ("b.name", P("b", "name")), ("c.name", P("c", "name")),
                ("e3.foo", ElementProperty(Var("e3", "RELATIONSHIP"), "foo", "ANY")))]),
     [{"a.name": "Alice", "b.name": "Eve", "c.name": "Paul", "e3.foo": 42},
      {"a.name": "Eve", "b.name": "Paul", "c.name": "Alice", "e3.foo": None},
      {"a.name": "Paul", "b.name": "Alice", "c.name": "Eve", "e3.foo": None},
      {"a.name": "Bob", "b.name": "Eve", "c.name": "Paul", "e3.foo": None}]))
OPTIONAL_CASES.append(
    ("optional_match_stacked_empty", "MTa/OptionalMatchTests.scala:404-421", "CREATE (s {val: 1})",
     Query([Match([NodeP("a")]),
            Match([NodeP("a"), NodeP("b", ("NonExistent",))], [RelP("r1", "a", "b")], optional=True),
            Match([NodeP("a"), NodeP("c", ("NonExistent",))], [RelP("r2", "a", "c")], optional=True)],
           [ret(("b", N("b")), ("c", N("c")))]),
     [{"b": None, "c": None}]))
OPTIONAL_CASES += [
    ("optional_match_leading_no_label", "MTa/OptionalMatchTests.scala:51-60", "CREATE (:A)",
     Query([Match([NodeP("n", ("B",))], optional=True)], [ret(("n", N("n")))]),
     [{"n": None}]),
    # the reference RETURNs * (b as a node); b's name stands for the node here
    ("optional_match_leading", "MTa/OptionalMatchTests.scala:423-444",
     """CREATE (p1:Person {name: "Alice"})
        CREATE (p2:Person {name: "Bob"})""",
     Query([Match([NodeP("a", ("Foo",))], optional=True), Match([NodeP("b", ("Person",))])],
           [ret(("a", N("a")), ("b.name", P("b", "name")))]),
     [{"a": None, "b.name": "Alice"}, {"a": None, "b.name": "Bob"}]),
]
CASES = CASES + OPTIONAL_CASES


# ------------------------------------------------------------ ReturnTests (MTa)
# Element results (rowToCypherMap) and the RETURN tail
# (ORDER BY / SKIP / LIMIT / DISTINCT, §8(f) rank 4).  A 6th tuple element
# holds options: {"ordered": True} compares the row LIST (ORDER BY cases —
# the reference compares Bags, the order is what those tests are about),
# {"row_count": k} checks only the number of rows (the reference counts the
# rows of the underlying table).  Node / relationship values are
# CypherNode / CypherRelationship (planner.py); ids are CreateQueryParser's.
from capf_amd.expr import (Add, Ands, BoolLit, Equals, ExistsPattern, GreaterThan, IntegerLit,  # noqa: E402
                           Not, Ors, Param, StringLit)
from capf_amd.planner import CypherNode, CypherRelationship  # noqa: E402


def R(v):
    from capf_amd.expr import Var
    return Var(v, "RELATIONSHIP")


def node(i, labels=(), **props):
    return CypherNode(i, frozenset(labels), tuple(sorted(props.items())))


def rel(i, s, t, typ, **props):
    return CypherRelationship(i, s, t, typ, tuple(sorted(props.items())))


VALS3 = """CREATE (:Node {val: 4}), (:Node {val: 3}), (:Node  {val: 42})"""


def _val_query(**kw):
    return Query([Match([NodeP("a")])], [ret(("val", P("a", "val")), **kw)])


RETURN_CASES = [
    ("return_full_node", "MTa/ReturnTests.scala:103-112", "CREATE ({foo:'bar'}),()",
     scan_n(ret(("n", N("n")))),
     [{"n": node(0, foo="bar")}, {"n": node(1)}]),
    ("return_full_rel", "MTa/ReturnTests.scala:114-124", "CREATE ()-[:Rel {foo:'bar'}]->()-[:Rel]->()",
     Query([Match([NodeP("_a0"), NodeP("_a1")], [RelP("r", "_a0", "_a1")])], [ret(("r", R("r")))]),
     [{"r": rel(2, 0, 1, "Rel", foo="bar")}, {"r": rel(4, 1, 3, "Rel")}]),
    ("return_rel_property_untyped", "MTa/ReturnTests.scala:126-136", "CREATE ()-[:Rel {foo:'bar'}]->()-[:Rel]->()",
     Query([Match([NodeP("_a0"), NodeP("_a1")], [RelP("r", "_a0", "_a1")])],
           [ret(("r.foo", ElementProperty(R("r"), "foo", "STRING")))]),
     [{"r.foo": "bar"}, {"r.foo": None}]),
    ("return_multiple_references", "MTa/ReturnTests.scala:138-153", "CREATE ({val: 0})",
     Query([Match([NodeP("a")])],
           [ret(("a", N("a")), ("foo", P("a", "val"))), ret(("a", N("a")), ("bar", Var("foo"))),
            ret(("a.val", P("a", "val")))]),
     [{"a.val": 0}]),
    ("return_distinct_property", "MTa/ReturnTests.scala:157-174",
     """CREATE ({name:'bar'}) CREATE ({name:'bar'}) CREATE ({name:'baz'}) CREATE ({name:'baz'})
        CREATE ({name:'bar'}) CREATE ({name:'foo'})""",
     scan_n(ret(("name", P("n", "name")), distinct=True)),
     [{"name": "bar"}, {"name": "foo"}, {"name": "baz"}]),
    ("return_distinct_combinations", "MTa/ReturnTests.scala:176-193",
     """CREATE ({p1:'a', p2: 'a', p3: '1'}) CREATE ({p1:'a', p2: 'a', p3: '2'})
        CREATE ({p1:'a', p2: 'b', p3: '3'}) CREATE ({p1:'b', p2: 'a', p3: '4'})
        CREATE ({p1:'b', p2: 'b', p3: '5'})""",
     scan_n(ret(("p1", P("n", "p1")), ("p2", P("n", "p2")), distinct=True)),
     [{"p2": "a", "p1": "a"}, {"p2": "a", "p1": "b"}, {"p2": "b", "p1": "a"}, {"p2": "b", "p1": "b"}]),
    ("order_by_default", "MTa/ReturnTests.scala:196-207", VALS3,
     _val_query(order_by=[("val", "asc")]), [{"val": 3}, {"val": 4}, {"val": 42}], {"ordered": True}),
    ("order_by_asc", "MTa/ReturnTests.scala:209-220", VALS3,
     _val_query(order_by=[("val", "asc")]), [{"val": 3}, {"val": 4}, {"val": 42}], {"ordered": True}),
    ("order_by_desc", "MTa/ReturnTests.scala:222-233", VALS3,
     _val_query(order_by=[("val", "desc")]), [{"val": 42}, {"val": 4}, {"val": 3}], {"ordered": True}),
    ("skip", "MTa/ReturnTests.scala:236-243", VALS3, _val_query(skip=2), None, {"row_count": 1}),
    ("order_by_skip", "MTa/ReturnTests.scala:245-255", VALS3,
     _val_query(order_by=[("val", "asc")], skip=1), [{"val": 4}, {"val": 42}], {"ordered": True}),
    # SKIP 1 + 1: the front end folds the constant (Skip accepts a literal or parameter,
    # RelationalOperator.scala:362-377)
    ("order_by_arithmetic_skip", "MTa/ReturnTests.scala:257-267", VALS3,
     _val_query(order_by=[("val", "asc")], skip=IntegerLit(2)), [{"val": 42}], {"ordered": True}),
    ("limit", "MTa/ReturnTests.scala:270-277", VALS3, _val_query(limit=1), None, {"row_count": 1}),
    ("limit_parameter", "MTa/ReturnTests.scala:279-290", "CREATE (a:A),(b:B),(c:C)",
     Query([Match([NodeP("a")])], [ret(("a", N("a")), limit=Param("limit")), ret(("a", N("a")))]),
     None, {"row_count": 1, "params": {"limit": 1}}),
]

# ------------------------------------------- PredicateTests EXISTS (MTa :705-870)
# ExistsSubQuery (RelationalPlanner.scala:224-247), SURVEY §8(f) rank 3.


def _ex(nodes, rels, where=()):
    return ExistsPattern(Match(nodes, rels, list(where)))


EXISTS_CASES = [
    ("exists_basic", "MTa/PredicateTests.scala:706-722",
     """CREATE (v {id: 1})-[:REL]->({id: 2})-[:REL]->(w {id: 3})
        CREATE (v)-[:REL]->(w)
        CREATE (w)-[:REL]->({id: 4})""",
     Query([Match([NodeP("a"), NodeP("b")], [RelP("_r0", "a", "b")],
                  [_ex([NodeP("a"), NodeP("_x"), NodeP("b")], [RelP("_e1", "a", "_x"), RelP("_e2", "_x", "b")])])],
           [ret(("a.id", P("a", "id")), ("b.id", P("b", "id")))]),
     [{"a.id": 1, "b.id": 3}]),
    ("exists_var_length", "MTa/PredicateTests.scala:724-735",
     "CREATE (v {id: 1})-[:REL]->({id: 2})-[:REL]->({id: 3})<-[:REL]-(v)",
     Query([Match([NodeP("a"), NodeP("b")], [RelP("_r0", "a", "b")],
                  [_ex([NodeP("a"), NodeP("_x"), NodeP("b")],
                       [RelP("_e1", "a", "_x", length=(1, 3)), RelP("_e2", "_x", "b")])])],
           [ret(("a.id", P("a", "id")), ("b.id", P("b", "id")))]),
     [{"a.id": 1, "b.id": 3}]),
    ("exists_node_predicate", "MTa/PredicateTests.scala:737-751",
     """CREATE ({id: 1})-[:REL]->({name: 'foo'})
        CREATE ({id: 3})-[:REL]->({name: 'bar'})""",
     Query([Match([NodeP("a")], [],
                  [_ex([NodeP("a"), NodeP("_x")], [RelP("_e1", "a", "_x")],
                       [Equals(P("_x", "name"), StringLit("foo"))])])],
           [ret(("a.id", P("a", "id")))]),
     [{"a.id": 1}]),
    ("exists_rel_predicate", "MTa/PredicateTests.scala:753-767",
     """CREATE (v {id: 1})-[:REL {val: 'foo'}]->()-[:REL]->({id: 2})<-[:REL]-(v)
        CREATE (w {id: 3})-[:REL {val: 'bar'}]->()-[:REL]->({id: 4})<-[:REL]-(w)""",
     Query([Match([NodeP("a"), NodeP("b")], [RelP("_r0", "a", "b")],
                  [_ex([NodeP("a"), NodeP("_x"), NodeP("b")], [RelP("_e1", "a", "_x"), RelP("_e2", "_x", "b")],
                       [Equals(ElementProperty(R("_e1"), "val", "STRING"), StringLit("foo"))])])],
           [ret(("a.id", P("a", "id")), ("b.id", P("b", "id")))]),
     [{"a.id": 1, "b.id": 2}]),
    ("exists_label_predicate", "MTa/PredicateTests.scala:769-783",
     """CREATE (v{id: 1})-[:REL {val: 'foo'}]->(:A)-[:REL]->({id: 2})<-[:REL]-(v)
        CREATE (w{id: 3})-[:REL {val: 'bar'}]->(:B)-[:REL]->({id: 4})<-[:REL]-(w)""",
     Query([Match([NodeP("a"), NodeP("b")], [RelP("_r0", "a", "b")],
                  [_ex([NodeP("a"), NodeP("_x", ("A",)), NodeP("b")],
                       [RelP("_e1", "a", "_x"), RelP("_e2", "_x", "b")])])],
           [ret(("a.id", P("a", "id")), ("b.id", P("b", "id")))]),
     [{"a.id": 1, "b.id": 2}]),
    ("exists_type_predicate", "MTa/PredicateTests.scala:785-799",
     """CREATE (v {id: 1})-[:A]->()-[:REL]->({id: 2})<-[:REL]-(v)
        CREATE (w {id: 3})-[:B]->()-[:REL]->({id: 4})<-[:REL]-(w)""",
     Query([Match([NodeP("a"), NodeP("b")], [RelP("_r0", "a", "b")],
                  [_ex([NodeP("a"), NodeP("_x"), NodeP("b")],
                       [RelP("_e1", "a", "_x", ("A",)), RelP("_e2", "_x", "b")])])],
           [ret(("a.id", P("a", "id")), ("b.id", P("b", "id")))]),
     [{"a.id": 1, "b.id": 2}]),
    ("exists_inverse", "MTa/PredicateTests.scala:801-813",
     "CREATE (v {id: 1})-[:REL]->({id: 2})-[:REL]->({id: 3})<-[:REL]-(v)",
     Query([Match([NodeP("a"), NodeP("b")], [RelP("_r0", "a", "b")],
                  [Not(_ex([NodeP("a"), NodeP("_x"), NodeP("b")], [RelP("_e1", "a", "_x"), RelP("_e2", "_x", "b")]))])],
           [ret(("a.id", P("a", "id")), ("b.id", P("b", "id")))]),
     [{"a.id": 1, "b.id": 2}, {"a.id": 2, "b.id": 3}]),
    ("exists_nested", "MTa/PredicateTests.scala:815-838",
     """CREATE ({id: 1, age: 21})
        CREATE ({id: 2, age: 18, foo: true})
        CREATE ({id: 3, age: 18, foo: true})-[:KNOWS]->(:Foo)
        CREATE ({id: 4, age: 18, foo: false})-[:KNOWS]->(:Foo)""",
     Query([Match([NodeP("a")], [],
                  [Ors(GreaterThan(P("a", "age"), IntegerLit(20)),
                       Ands(_ex([NodeP("a"), NodeP("_x", ("Foo",))], [RelP("_e1", "a", "_x", ("KNOWS",))]),
                            Equals(P("a", "foo"), BoolLit(True))))])],
           [ret(("a.id", P("a", "id")))]),
     [{"a.id": 1}, {"a.id": 3}]),
    ("exists_derived_node_predicate", "MTa/PredicateTests.scala:840-856",
     """CREATE ({id: 1, val: 0})-[:REL]->({id: 3, val: 2})
        CREATE ({id: 2, val: 0})-[:REL]->({id: 3, val: 1})""",
     Query([Match([NodeP("a")], [],
                  [_ex([NodeP("a"), NodeP("_x")], [RelP("_e1", "a", "_x")],
                       [Equals(P("_x", "val"), Add(P("a", "val"), IntegerLit(2)))])])],
           [ret(("a.id", P("a", "id")))]),
     [{"a.id": 1}]),
    ("exists_multiple_predicates", "MTa/PredicateTests.scala:858-869",
     "CREATE ({id: 1})-[:REL]->({id: 2, foo: true})",
     Query([Match([NodeP("a")], [],
                  [_ex([NodeP("a"), NodeP("_x")], [RelP("_e1", "a", "_x")],
                       [Equals(P("_x", "id"), IntegerLit(2)), Equals(P("_x", "foo"), BoolLit(True))])])],
           [ret(("a.id", P("a", "id")))]),
     [{"a.id": 1}]),
]

# The two pattern-predicate sections before it (:373-537 `WHERE (a)-->()-->(b)`,
# :538-704 the same under "Inline pattern predicates") hold the same graphs,
# queries and Bags as the EXISTS(...) section; the front end turns a pattern in
# WHERE into that section's ExistsPattern, so they are its plans under their
# own sources.
_PP_STARTS = {"pattern": (373, 391, 404, 421, 438, 455, 472, 486, 508, 525, 537),
              "inline": (539, 557, 570, 587, 604, 621, 638, 652, 674, 691, 703)}
PATTERN_PREDICATE_CASES = [
    (c[0].replace("exists_", f"{tag}_pred_"), f"MTa/PredicateTests.scala:{st[i]}-{st[i + 1] - 1}", *c[2:])
    for tag, st in _PP_STARTS.items() for i, c in enumerate(EXISTS_CASES)]
CASES = CASES + RETURN_CASES + EXISTS_CASES + PATTERN_PREDICATE_CASES


# ------------------------------- AggregationTests "in WITH" / "without alias" (FTt)
# WITH agg AS res RETURN res: the aggregate is a WITH stage, RETURN projects
# its alias (a second projection over the grouped table).


def _in_with(alias, agg):
    return scan_n(ret((alias, agg)), ret((alias, Var(alias))))


SIX_NAMES = "CREATE ({name: 'foo'}), ({name: 'bar'}), (), (), (), ({name: 'baz'})"
AGG_WITH_CASES = [
    ("avg_ints_with", "FTt/acceptance/AggregationTests.scala:39-47", INTS,
     _in_with("res", Avg(P("n", "val"))), [{"res": 4}], {"coop": True}),
    ("avg_ints_no_alias", "FTt/acceptance/AggregationTests.scala:59-67", INTS,
     scan_n(ret(("AVG(n.val)", Avg(P("n", "val"))))), [{"AVG(n.val)": 4}], {"coop": True}),
    ("avg_floats_with", "FTt/acceptance/AggregationTests.scala:69-77", FLOATS,
     _in_with("res", Avg(P("n", "val"))), [{"res": 3.5}]),
    ("avg_single_null_with", "FTt/acceptance/AggregationTests.scala:89-97", FLOATS_NULL,
     _in_with("res", Avg(P("n", "val"))), [{"res": 32.5}]),
    ("avg_only_nulls_with", "FTt/acceptance/AggregationTests.scala:109-117", NULLS,
     _in_with("res", Avg(P("n", "val"))), [{"res": None}]),
    ("count_star_with", "FTt/acceptance/AggregationTests.scala:140-148", SIX_NAMES,
     _in_with("nbrRows", CountStar()), [{"nbrRows": 6}]),
    ("count_n_no_alias", "FTt/acceptance/AggregationTests.scala:170-178", SIX_NAMES,
     scan_n(ret(("count(n)", Count(N("n"))))), [{"count(n)": 6}]),
    ("count_star_no_alias", "FTt/acceptance/AggregationTests.scala:180-188", SIX_NAMES,
     scan_n(ret(("count(*)", CountStar()))), [{"count(*)": 6}]),
    ("count_node_with", "FTt/acceptance/AggregationTests.scala:200-208", SIX_NAMES,
     _in_with("nodes", Count(N("n"))), [{"nodes": 6}]),
    ("count_grouping_with", "FTt/acceptance/AggregationTests.scala:232-242",
     "CREATE ({name: 'foo'}), ({name: 'foo'}), (), (), (), ({name: 'baz'})",
     scan_n(ret(("name", P("n", "name")), ("amount", CountStar())),
            ret(("name", Var("name")), ("amount", Var("amount")))),
     [{"name": "foo", "amount": 2}, {"name": None, "amount": 3}, {"name": "baz", "amount": 1}]),
    ("min_with", "FTt/acceptance/AggregationTests.scala:282-290", INTS3,
     _in_with("res", Min(P("n", "val"))), [{"res": 23}]),
    ("min_single_null_with", "FTt/acceptance/AggregationTests.scala:302-310", INTS_NULL,
     _in_with("res", Min(P("n", "val"))), [{"res": 23}]),
    ("min_single_null_no_alias", "FTt/acceptance/AggregationTests.scala:322-330", INTS_NULL,
     scan_n(ret(("MIN(n.val)", Min(P("n", "val"))))), [{"MIN(n.val)": 23}]),
    ("min_only_nulls_with", "FTt/acceptance/AggregationTests.scala:332-340", NULLS,
     _in_with("res", Min(P("n", "val"))), [{"res": None}]),
    ("max_with", "FTt/acceptance/AggregationTests.scala:387-395", INTS3,
     _in_with("res", Max(P("n", "val"))), [{"res": 84}]),
    ("max_single_null_with", "FTt/acceptance/AggregationTests.scala:407-415", INTS_NULL,
     _in_with("res", Max(P("n", "val"))), [{"res": 42}]),
    ("max_single_null_no_alias", "FTt/acceptance/AggregationTests.scala:427-435", INTS_NULL,
     scan_n(ret(("MAX(n.val)", Max(P("n", "val"))))), [{"MAX(n.val)": 42}]),
    ("max_only_nulls_with", "FTt/acceptance/AggregationTests.scala:437-445", NULLS,
     _in_with("res", Max(P("n", "val"))), [{"res": None}]),
    ("sum_ints_with", "FTt/acceptance/AggregationTests.scala:494-502", INTS,
     _in_with("res", Sum(P("n", "val"))), [{"res": 12}]),
    ("sum_floats_with", "FTt/acceptance/AggregationTests.scala:514-522", FLOATS,
     _in_with("res", Sum(P("n", "val"))), [{"res": 10.5}]),
    ("sum_floats_no_alias", "FTt/acceptance/AggregationTests.scala:534-542", FLOATS,
     scan_n(ret(("SUM(n.val)", Sum(P("n", "val"))))), [{"SUM(n.val)": 10.5}]),
    ("sum_single_null_with", "FTt/acceptance/AggregationTests.scala:544-552", FLOATS_NULL,
     _in_with("res", Sum(P("n", "val"))), [{"res": 65.0}]),
    ("sum_only_nulls_with", "FTt/acceptance/AggregationTests.scala:564-572", NULLS,
     _in_with("res", Sum(P("n", "val"))), [{"res": None}]),
]
CASES = CASES + AGG_WITH_CASES


# ------------------------------ AggregationTests COLLECT / Combinations (FTt)
# collect(e) is Flink's COLLECT, a MULTISET (FlinkSQLExprMapper.scala:283): the
# reference compares the lists with .toBag, and so does conftest.bag.
# avg over INTEGER values is a FLOAT (49.666…, 32.5), as these reference tests
# expect; option "typed" marks the cases whose reference test compares the
# CypherValues directly (`rows.head("avg") should equal(CypherFloat(…))`).


def _agg_all():
    return [("avg", Avg(P("n", "val"))), ("cnt", CountStar()), ("min", Min(P("n", "val"))),
            ("max", Max(P("n", "val"))), ("sum", Sum(P("n", "val"))), ("col", Collect(P("n", "val")))]


COMB_OUT = ["avg", "cnt", "min", "max", "sum", "col"]
KEYED_INTS = "CREATE ({key: 'a', val: 42}),({key: 'a',val: 23}),({key: 'b', val: 84})"
KEYED_FLOATS = "CREATE ({key: 'a', val: 42.0}),({key: 'a',val: 23.0}),({key: 'b', val: 84.0})"

COLLECT_CASES = [
    ("collect_ints_with", "FTt/acceptance/AggregationTests.scala:734-743", INTS,
     _in_with("res", Collect(P("n", "val"))), [{"res": [2, 4, 6]}]),
    ("collect_ints_return", "FTt/acceptance/AggregationTests.scala:745-753", INTS,
     scan_n(ret(("res", Collect(P("n", "val"))))), [{"res": [2, 4, 6]}]),
    ("collect_single_null_with", "FTt/acceptance/AggregationTests.scala:755-763", FLOATS_NULL,
     _in_with("res", Collect(P("n", "val"))), [{"res": [23.0, 42.0]}]),
    ("collect_single_null_return", "FTt/acceptance/AggregationTests.scala:765-773", FLOATS_NULL,
     scan_n(ret(("res", Collect(P("n", "val"))))), [{"res": [23.0, 42.0]}]),
    ("collect_only_nulls_with", "FTt/acceptance/AggregationTests.scala:775-783", NULLS,
     _in_with("res", Collect(P("n", "val"))), [{"res": []}]),
    ("collect_only_nulls_return", "FTt/acceptance/AggregationTests.scala:785-793", NULLS,
     scan_n(ret(("res", Collect(P("n", "val"))))), [{"res": []}]),
    ("collect_distinct_grouping", "FTt/acceptance/AggregationTests.scala:795-815",
     "CREATE (a:Start{id: 1}) CREATE (a)-[:REL]->({val: \"foo\"}) CREATE (a)-[:REL]->({val: \"foo\"})",
     Query([Match([NodeP("a", ("Start",)), NodeP("b")], [RelP("_r", "a", "b")])],
           [ret(("a.id", P("a", "id")), ("val", Collect(P("b", "val"), distinct=True)))]),
     [{"a.id": 1, "val": ["foo"]}]),
    ("collect_absent_strings", "FTt/acceptance/AggregationTests.scala:817-831",
     "CREATE (a:Person{id: 1, name:'Anna'}) CREATE (b:Person{id: 2, name:'Bob'}) "
     "CREATE (p1:Purchase{id: 3}) CREATE (a)-[:BOUGHT]->(p1)",
     Query([Match([NodeP("person", ("Person",)), NodeP("friend", ("Person",)), NodeP("customer", ("Customer",)),
                   NodeP("product", ("Product",))],
                  [RelP("_f", "person", "friend", ("FRIEND_OF",), "both"),
                   RelP("_i", "friend", "customer", ("IS",)),
                   RelP("_b", "customer", "product", ("BOUGHT",))])],
           [ret(("for", P("person", "name")),
                ("recommendations", Collect(P("product", "title"), distinct=True)))]),
     [], {"row_count": 0}),
    ("comb_with", "FTt/acceptance/AggregationTests.scala:835-857", INTS3,
     scan_n(ret(*_agg_all()), ret(*[(a, Var(a)) for a in COMB_OUT])),
     [{"avg": 49.666666666666664, "cnt": 3, "min": 23, "max": 84, "sum": 149, "col": [23, 42, 84]}],
     {"typed": True}),
    ("comb_return", "FTt/acceptance/AggregationTests.scala:859-880", INTS3,
     scan_n(ret(*_agg_all())),
     [{"avg": 49.666666666666664, "cnt": 3, "min": 23, "max": 84, "sum": 149, "col": [23, 42, 84]}],
     {"typed": True}),
    ("comb_grouping_return", "FTt/acceptance/AggregationTests.scala:882-901", KEYED_FLOATS,
     scan_n(ret(("key", P("n", "key")), *_agg_all())),
     [{"key": "b", "avg": 84.0, "cnt": 1, "min": 84.0, "max": 84.0, "sum": 84.0, "col": [84.0]},
      {"key": "a", "avg": 32.5, "cnt": 2, "min": 23.0, "max": 42.0, "sum": 65.0, "col": [23.0, 42.0]}]),
    ("comb_grouping_with", "FTt/acceptance/AggregationTests.scala:903-925", KEYED_INTS,
     scan_n(ret(("key", P("n", "key")), *_agg_all()),
            ret(*[(a, Var(a)) for a in ["key"] + COMB_OUT])),
     [{"key": "a", "avg": 32.5, "cnt": 2, "min": 23, "max": 42, "sum": 65, "col": [23, 42]},
      {"key": "b", "avg": 84.0, "cnt": 1, "min": 84, "max": 84, "sum": 84, "col": [84]}]),
]
CASES = CASES + COLLECT_CASES

# --------------------------------- ExpandIntoTests "Expand into after var expand"
CASES.append(
    ("expand_into_after_var_expand", "MTa/ExpandIntoTests.scala:109-145",
     """CREATE (p1:Person {name: "Alice"})
        CREATE (p2:Person {name: "Bob"})
        CREATE (comment:Comment)
        CREATE (post1:Post {content: "asdf"})
        CREATE (post2:Post {content: "foobar"})
        CREATE (p1)-[:KNOWS]->(p2)
        CREATE (p2)<-[:HASCREATOR]-(comment)
        CREATE (comment)-[:REPLYOF]->(post1)-[:REPLYOF]->(post2)
        CREATE (post2)-[:HASCREATOR]->(p1)""",
     Query([Match([NodeP("p1", ("Person",)), NodeP("p2", ("Person",)), NodeP("comment", ("Comment",)),
                   NodeP("post", ("Post",))],
                  [RelP("e1", "p1", "p2", ("KNOWS",)),
                   RelP("e2", "comment", "p2", ("HASCREATOR",)),
                   RelP("e3", "comment", "post", ("REPLYOF",), length=(1, 10)),
                   RelP("_h", "post", "p1", ("HASCREATOR",))],
                  where=[Equals(P("p1", "name"), StringLit("Alice"))])],
           [ret(("p1.name", P("p1", "name")), ("p2.name", P("p2", "name")),
                ("post.content", P("post", "content")))]),
     [{"p1.name": "Alice", "p2.name": "Bob", "post.content": "foobar"}]))


# ------------------------- expressions: id / exists / type / size / IN (MTa, FlinkSQLExprMapper :80-134)
def _r(v):
    return Var(v, "RELATIONSHIP")


def _unit(*items):
    return Query([], [ret(*items)])


A3 = "CREATE (:A {val: 1}), (:A {val: 2}), (:A {val: 3})"
EXPR_CASES = [
    ("fn_exists", "MTa/FunctionTests.scala:596-608", "CREATE ({id: 1}), ({id: 2}), ({other: 'foo'}), ()",
     scan_n(ret(("exists", Exists(P("n", "id"))))),
     [{"exists": True}, {"exists": True}, {"exists": False}, {"exists": False}]),
    ("fn_type", "MTa/FunctionTests.scala:635-647", "CREATE ()-[:KNOWS]->()-[:HATES]->()-[:REL]->()",
     Query([Match([NodeP("_a"), NodeP("_b")], [RelP("r", "_a", "_b")])], [ret(("type(r)", Type(_r("r"))))]),
     [{"type(r)": "KNOWS"}, {"type(r)": "HATES"}, {"type(r)": "REL"}]),
    # the reference encodes the ids as Morpheus ids; CAPF's are the raw LONGs
    ("fn_id_node", "MTa/FunctionTests.scala:651-657", "CREATE (),()",
     scan_n(ret(("id(n)", Id(N("n"))))), [{"id(n)": 0}, {"id(n)": 1}]),
    ("fn_id_rel", "MTa/FunctionTests.scala:659-665", "CREATE ()-[:REL]->()-[:REL]->()",
     Query([Match([NodeP("_a"), NodeP("_b")], [RelP("e", "_a", "_b")])], [ret(("id(e)", Id(_r("e"))))]),
     [{"id(e)": 2}, {"id(e)": 4}]),
    ("fn_size_literal_list", "MTa/FunctionTests.scala:722-731", "CREATE ()",
     scan_n(ret(("s", Size(ListLit(StringLit("Alice"), StringLit("Bob")))))), [{"s": 2}]),
    ("fn_size_literal_string", "MTa/FunctionTests.scala:733-742", "CREATE ()",
     scan_n(ret(("s", Size(StringLit("Alice"))))), [{"s": 5}]),
    ("fn_size_retrieved_string", "MTa/FunctionTests.scala:744-753", "CREATE ({name: 'Alice'})",
     Query([Match([NodeP("a")])], [ret(("s", Size(P("a", "name", "STRING"))))]), [{"s": 5}]),
    ("fn_size_null", "MTa/FunctionTests.scala:769-779", "CREATE ()",
     Query([Match([NodeP("a")])], [ret(("s", Size(P("a", "prop"))))]), [{"s": None}]),
    ("pred_in", "MTa/PredicateTests.scala:56-67", A3,
     Query([Match([NodeP("a", ("A",))], where=[In(P("a", "val"), ListLit(IntegerLit(-1), IntegerLit(2),
                                                                          IntegerLit(5), IntegerLit(0)))])],
           [ret(("a.val", P("a", "val")))]), [{"a.val": 2}]),
    ("pred_in_param", "MTa/PredicateTests.scala:69-80", A3,
     Query([Match([NodeP("a", ("A",))], where=[In(P("a", "val"), Param("list"))])],
           [ret(("a.val", P("a", "val")))]), [{"a.val": 2}], {"params": {"list": [-1, 2, 5, 0]}}),
    ("null_in_empty", "MTa/NullTests.scala:127", "",
     _unit(("res", In(NullLit(), ListLit()))), [{"res": False}]),
    ("null_in_list", "MTa/NullTests.scala:128", "",
     _unit(("res", In(NullLit(), ListLit(IntegerLit(1), IntegerLit(2))))), [{"res": None}]),
    ("null_in_null", "MTa/NullTests.scala:129", "",
     _unit(("res", In(NullLit(), ListLit(NullLit())))), [{"res": None}]),
    ("null_in_list_null", "MTa/NullTests.scala:130", "",
     _unit(("res", In(NullLit(), ListLit(IntegerLit(1), NullLit())))), [{"res": None}]),
    ("one_in_list_null", "MTa/NullTests.scala:131", "",
     _unit(("res", In(IntegerLit(1), ListLit(IntegerLit(1), NullLit())))), [{"res": True}]),
    ("two_in_list_null", "MTa/NullTests.scala:132", "",
     _unit(("res", In(IntegerLit(2), ListLit(IntegerLit(1), NullLit())))), [{"res": None}]),
    ("null_id", "MTa/NullTests.scala:47", "", _unit(("res", Id(NullLit()))), [{"res": None}]),
    ("null_type", "MTa/NullTests.scala:49", "", _unit(("res", Type(NullLit()))), [{"res": None}]),
]
CASES = CASES + EXPR_CASES


# ------------------- AggregationTests stDev / stDevP / percentiles (FTt :593-730)
# UNWIND <list literal> AS x is the relational `add(Explode(list) as x)`
# (RelationalPlanner.scala:99-101) over the unit table; round(agg * 1000) /
# 1000.0 aggregates first, then projects (okapi plans the Aggregate below the
# Project).  stDev / stDevP are Flink's stddevSamp / stddevPop
# (FlinkSQLExprMapper.scala:223-224); the percentiles follow the Spark
# backend's UDAFs (PercentileUdafs.scala:59-96) — Flink has no mapping.
def _unwind(values, alias, *items):
    from capf_amd.planner import Unwind
    lit = ListLit(*[NullLit() if v is None else FloatLit(v) if isinstance(v, float) else IntegerLit(v)
                    for v in values])
    return Query([Unwind(lit, alias)], [ret(*items)])


def _round3(agg):
    from capf_amd.expr import Divide, FloatLit as F, Multiply, Round
    return Divide(Round(Multiply(agg, IntegerLit(1000))), F(1000.0))


STDEV5 = [98.17, 112.3, 102.6, 94.3, 108.1]
STDEV5N = [98.17, None, 102.6, 94.3, 108.1]


def _stat_cases():
    from capf_amd.expr import PercentileCont, PercentileDisc, StDev, StDevP
    x = lambda v: Var(v)  # noqa: E731
    src = "FTt/acceptance/AggregationTests.scala:"
    return [
        ("stdev_floats", src + "594-600", "",
         _unwind(STDEV5, "numbers", ("res", _round3(StDev(x("numbers"))))), [{"res": 7.274}]),
        ("stdev_nullable_floats", src + "602-608", "",
         _unwind(STDEV5N, "numbers", ("res", _round3(StDev(x("numbers"))))), [{"res": 5.936}]),
        ("stdev_null", src + "610-617", "", _unit(("res", StDev(NullLit()))), [{"res": None}]),
        ("stdevp_floats", src + "621-627", "",
         _unwind(STDEV5, "numbers", ("res", _round3(StDevP(x("numbers"))))), [{"res": 6.506}]),
        ("stdevp_nullable_floats", src + "629-635", "",
         _unwind(STDEV5N, "numbers", ("res", _round3(StDevP(x("numbers"))))), [{"res": 5.140}]),
        ("stdevp_null", src + "637-644", "", _unit(("res", StDevP(NullLit()))), [{"res": None}]),
        ("pcont_ints", src + "648-654", "",
         _unwind([1, 2], "values", ("res", PercentileCont(x("values"), FloatLit(0.5)))), [{"res": 1.5}]),
        ("pcont_one", src + "656-662", "",
         _unwind([2, 10, 5, 6], "values", ("res", PercentileCont(x("values"), FloatLit(1.0)))), [{"res": 10.0}]),
        ("pcont_zero", src + "664-670", "",
         _unwind([2, 10, 5, 6], "values", ("res", PercentileCont(x("values"), FloatLit(0.0)))), [{"res": 2.0}]),
        ("pcont_floats_null", src + "672-678", "",
         _unwind([10.0, None, 2.0, 6.0], "values", ("res", _round3(PercentileCont(x("values"), FloatLit(0.62))))),
         [{"res": 6.96}]),
        ("pcont_floats", src + "680-686", "",
         _unwind([10.0, 5.0, 2.0, 6.0], "values", ("res", PercentileCont(x("values"), FloatLit(0.6)))),
         [{"res": 5.8}]),
        ("pdisc_ints", src + "690-696", "",
         _unwind([10, 5, 2, 6], "values", ("res", PercentileDisc(x("values"), FloatLit(0.5)))), [{"res": 5}]),
        ("pdisc_one", src + "698-704", "",
         _unwind([10.0, 5.0, 2.0, 6.0], "values", ("res", PercentileDisc(x("values"), FloatLit(1.0)))),
         [{"res": 10.0}]),
        ("pdisc_zero", src + "706-712", "",
         _unwind([10.0, 5.0, 2.0, 6.0], "values", ("res", PercentileDisc(x("values"), FloatLit(0.0)))),
         [{"res": 2.0}]),
        ("pdisc_floats_null", src + "714-720", "",
         _unwind([10.0, None, 2.0, 6.0], "values", ("res", PercentileDisc(x("values"), FloatLit(0.6)))),
         [{"res": 6.0}]),
        ("pdisc_floats_graph", src + "722-729", "CREATE ({age: 10.0}), ({age: 2.0}), ({age: 5.0}), ({age: 6.0})",
         scan_n(ret(("res", PercentileDisc(P("n", "age"), FloatLit(0.5))))), [{"res": 5.0}]),
    ]


STAT_CASES = _stat_cases()
CASES = CASES + STAT_CASES


# ------------------------------------------ FunctionTests (MTa), VERDICT r5 item 3
from function_cases import FUNCTION_CASES  # noqa: E402

CASES = CASES + FUNCTION_CASES

# ----------------------- NullTests / ExpressionTests (MTa), VERDICT r5 items 3, 7
from expression_cases import EXPRESSION_CASES  # noqa: E402

CASES = CASES + EXPRESSION_CASES

# ------------------- MatchTests / UnwindTests / WithTests / ReturnTests / OptionalMatchTests (MTa)
from clause_cases import CLAUSE_CASES, ERROR_CASES  # noqa: E402,F401

CASES = CASES + CLAUSE_CASES
