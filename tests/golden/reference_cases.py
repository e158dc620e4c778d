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
from capf_amd.expr import (Avg, Count, CountStar, ElementProperty, Max, Min, Sum, Var)
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
    ("avg_ints", "FTt/acceptance/AggregationTests.scala:49-57", INTS,
     scan_n(ret(("res", Avg(P("n", "val"))))), [{"res": 4}]),
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
