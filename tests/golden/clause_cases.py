"""Clause cases transcribed from the shared-planner acceptance suite (MTa =
morpheus-testing/src/test/scala/org/opencypher/morpheus/impl/acceptance/):
MatchTests, UnwindTests, WithTests, the rest of ReturnTests and
OptionalMatchTests.  Same format as reference_cases.py; each plan is the okapi
IR the front end builds for the test's query (a pattern in one MATCH is one
Match; `(a)--(b)` is direction "both"; `WITH ... UNWIND` an Unwind among the
stages; `RETURN 1` a leading stage over the unit table).

Not transcribed: MatchTests :420-431 (CONSTRUCT, a catalog feature),
OptionalMatchTests :93-120 (a Spark session setting), ReturnTests :333-337
(Spark DataFrame struct access) and :344-356 (a LIST of MAPs: MAP values are a
struct of columns here, and LIST columns hold scalars), UnwindTests :118-132
(`ignore`d upstream), PatternScanTests (pre-joined pattern tables are a Spark
graph-storage feature; the query results are the plain MATCH results).  The
MatchTests schema conflicts (:380-418) expect an exception, not a Bag:
ERROR_CASES.
"""
import capf_import  # noqa: F401
from capf_amd.expr import (Add, Ands, BoolLit, Collect, Count, ElementProperty, Equals, GreaterThan, GreaterThanOrEqual, Id,
                           IntegerLit, LessThanOrEqual, ListLit, MapExpression, Not, NullLit, Param, StringLit, Type,
                           Var)
from capf_amd.planner import CypherNode, CypherRelationship, Match, NodeP, Query, RelP, Stage, UnionQuery, Unwind

MT = "MTa/MatchTests.scala:"
UT = "MTa/UnwindTests.scala:"
WT = "MTa/WithTests.scala:"
RT = "MTa/ReturnTests.scala:"
OT = "MTa/OptionalMatchTests.scala:"
NT = "MTa/UnionTests.scala:"


def ret(*items, **kw):
    return Stage(list(items), **kw)


def P(v, k):
    return ElementProperty(Var(v, "NODE"), k)


def N(v):
    return Var(v, "NODE")


def node(i, labels=(), **props):
    return CypherNode(i, frozenset(labels), tuple(sorted(props.items())))


def _ints(*xs):
    return ListLit(*[IntegerLit(x) for x in xs])


SPRAWL = """CREATE (a:Person {name: "Philip"})
            CREATE (b:Person {name: "Stefan"})
            CREATE (c:City {name: "The Pan-European Sprawl"})
            CREATE (a)-[:KNOWS]->(b)
            CREATE (a)-[:LIVES_IN]->(c)
            CREATE (b)-[:LIVES_IN]->(c)"""
NARCISSISTS = """CREATE (p1:Narcissist {name: "Alice"})
                 CREATE (p2:Narcissist {name: "Bob"})
                 CREATE (p1)-[:LOVES]->(p1)
                 CREATE (p2)-[:LOVES]->(p2)"""


def _match_cases():
    ab = Match([NodeP("a", ("Narcissist",)), NodeP("b", ("Narcissist",))])
    one_two = [ret(("one", P("a", "name")), ("two", P("b", "name")))]
    return [
        ("match_empty_graph", MT + "41-49", "", Query([Match([NodeP("n")])], [ret(("n", N("n")))]), []),
        ("match_missing_label", MT + "51-60", "CREATE (:A)",
         Query([Match([NodeP("n", ("B",))])], [ret(("n", N("n")))]), []),
        ("match_empty_scan_graph", MT + "62-71", "", Query([Match([NodeP("n")])], [ret(("n", N("n")))]), []),
        ("match_label", MT + "76-93", 'CREATE (p:Person {firstName: "Alice", lastName: "Foo"})',
         Query([Match([NodeP("a", ("Person",))])], [ret(("a.firstName", P("a", "firstName")))]),
         [{"a.firstName": "Alice"}]),
        ("match_unknown_label", MT + "95-108", "CREATE (p:Person {firstName: 'Alice', lastName: 'Foo'})",
         Query([Match([NodeP("a", ("Animal",))])], [ret(("a", N("a")))]), []),
        ("match_multiple_clauses", MT + "112-140",
         """CREATE (p1:Person {name: "Alice"})
            CREATE (p2:Person {name: "Bob"})
            CREATE (p3:Person {name: "Eve"})
            CREATE (p1)-[:KNOWS]->(p2)
            CREATE (p2)-[:KNOWS]->(p3)""",
         Query([Match([NodeP("p1", ("Person",))]),
                Match([NodeP("p1", ("Person",)), NodeP("p2", ("Person",))], [RelP("e1", "p1", "p2")]),
                Match([NodeP("p2"), NodeP("p3", ("Person",))], [RelP("e2", "p2", "p3")])],
               [ret(("p1.name", P("p1", "name")), ("p2.name", P("p2", "name")), ("p3.name", P("p3", "name")))]),
         [{"p1.name": "Alice", "p2.name": "Bob", "p3.name": "Eve"}]),
        ("match_disconnected_components", MT + "181-206", NARCISSISTS, Query([ab], one_two),
         [{"one": "Alice", "two": "Alice"}, {"one": "Alice", "two": "Bob"}, {"one": "Bob", "two": "Bob"},
          {"one": "Bob", "two": "Alice"}]),
        ("match_joined_components", MT + "208-234", NARCISSISTS,
         Query([Match(ab.nodes, [], [Equals(P("a", "name"), P("b", "name"))])], one_two),
         [{"one": "Alice", "two": "Alice"}, {"one": "Bob", "two": "Bob"}]),
        ("match_cross_product_clauses", MT + "236-249", "CREATE (:A {val: 0}), (:B {val: 1})-[:REL]->(:C {val: 2})",
         Query([Match([NodeP("a", ("A",))]),
                Match([NodeP("b", ("B",)), NodeP("c", ("C",))], [RelP("_r", "b", "c")])],
               [ret(("a.val", P("a", "val")), ("c.val", P("c", "val")))]),
         [{"a.val": 0, "c.val": 2}]),
        ("match_undirected", MT + "252-271",
         """CREATE (a:A {prop: 'isA'})
            CREATE (b:B {prop: 'fromA'})
            CREATE (c:C {prop: 'toA'})
            CREATE (d:D)
            CREATE (a)-[:T]->(b)
            CREATE (b)-[:T]->(c)
            CREATE (c)-[:T]->(a)""",
         Query([Match([NodeP("a", ("A",)), NodeP("other")], [RelP("_r", "a", "other", direction="both")])],
               [ret(("a.prop", P("a", "prop")), ("other.prop", P("other", "prop")))]),
         [{"a.prop": "isA", "other.prop": "fromA"}, {"a.prop": "isA", "other.prop": "toA"}]),
        ("match_undirected_prebound", MT + "296-316",
         """CREATE (a:A {prop: 'a'})
            CREATE (b:B {prop: 'b'})
            CREATE (b)-[:T]->(a)
            CREATE (a)-[:T]->(b)""",
         Query([Match([NodeP("a", ("A",))]), Match([NodeP("b", ("B",))]),
                Match([NodeP("a"), NodeP("b")], [RelP("_r", "a", "b", direction="both")])],
               [ret(("a.prop", P("a", "prop")), ("b.prop", P("b", "prop")))]),
         [{"a.prop": "a", "b.prop": "b"}, {"a.prop": "a", "b.prop": "b"}]),
        # (a)--(a): an undirected self-loop matches once per rel (2 loops × {a's
        # other loop, b→a} = 4 rows, not 8)
        ("match_mixed_directed_undirected", MT + "320-341",
         """CREATE (a:A {prop: 'a'})
            CREATE (b:B {prop: 'b'})
            CREATE (c:C {prop: 'c'})
            CREATE (a)-[:T]->(a)
            CREATE (a)-[:T]->(a)
            CREATE (b)-[:T]->(a)
            CREATE (a)-[:T]->(c)""",
         Query([Match([NodeP("a", ("A",)), NodeP("other")],
                      [RelP("_r1", "a", "a", direction="both"), RelP("_r2", "other", "a")])],
               [ret(("a.prop", P("a", "prop")), ("other.prop", P("other", "prop")))]),
         [{"a.prop": "a", "other.prop": "a"}, {"a.prop": "a", "other.prop": "a"},
          {"a.prop": "a", "other.prop": "b"}, {"a.prop": "a", "other.prop": "b"}]),
        ("match_expand_into_var_length", MT + "443-454", SPRAWL,
         Query([Match([NodeP("a", ("Person",)), NodeP("c", ("City",)), NodeP("b", ("Person",))],
                      [RelP("_r1", "a", "c", ("LIVES_IN",)), RelP("_r2", "b", "c", ("LIVES_IN",)),
                       RelP("_r3", "a", "b", ("KNOWS",), length=(1, 2))])],
               [ret(("a.name", P("a", "name")), ("b.name", P("b", "name")), ("c.name", P("c", "name")))]),
         [{"a.name": "Philip", "b.name": "Stefan", "c.name": "The Pan-European Sprawl"}]),
        ("match_type_disjunction", MT + "458-466", SPRAWL,
         Query([Match([NodeP("_a"), NodeP("_b")], [RelP("r", "_a", "_b", ("LIVES_IN", "KNOWS"))])],
               [ret(("type(r)", Type(Var("r", "RELATIONSHIP"))))]),
         [{"type(r)": "LIVES_IN"}, {"type(r)": "LIVES_IN"}, {"type(r)": "KNOWS"}]),
        ("match_type_disjunction_var_length", MT + "468-491",
         """CREATE (a { val: 'a' })
            CREATE (b { val: 'b' })
            CREATE (c { val: 'c' })
            CREATE (d { val: 'd' })
            CREATE (a)-[:A]->(a)
            CREATE (a)-[:B]->(b)
            CREATE (b)-[:C]->(c)
            CREATE (c)-[:D]->(d)""",
         Query([Match([NodeP("from"), NodeP("to")], [RelP("_r", "from", "to", ("A", "B", "C", "D"), length=(1, 3))])],
               [ret(("from", P("from", "val")), ("to", P("to", "val")))]),
         [{"from": "a", "to": "a"}, {"from": "a", "to": "b"}, {"from": "a", "to": "b"}, {"from": "a", "to": "c"},
          {"from": "a", "to": "c"}, {"from": "a", "to": "d"}, {"from": "b", "to": "c"}, {"from": "b", "to": "d"},
          {"from": "c", "to": "d"}]),
    ]


def _unwind_cases():
    par = {"params": {"param": [1, 2, 3]}}
    chain = "CREATE (:A)-[:T]->(:B {item: '1'})-[:T]->(:C)"
    arb = Match([NodeP("a"), NodeP("b")], [RelP("r", "a", "b")])
    na, nb = node(0, ("A",)), node(1, ("B",), item="1")
    # a LIST property column is not routed between ranks
    lo = {"local_only": True}
    return [
        ("unwind_parameter", UT + "36-47", "", Query([Unwind(Param("param"), "item")], [ret(("item", Var("item")))]),
         [{"item": 1}, {"item": 2}, {"item": 3}], par),
        ("unwind_literal", UT + "49-61", "", Query([Unwind(_ints(1, 2, 3), "item")], [ret(("item", Var("item")))]),
         [{"item": 1}, {"item": 2}, {"item": 3}]),
        ("unwind_after_match", UT + "63-80", chain,
         Query([arb, Unwind(Param("param"), "item")], [ret(("a", N("a")), ("item", Var("item")))]),
         [{"a": a, "item": i} for a in (na, nb) for i in (1, 2, 3)], par),
        ("unwind_collected", UT + "82-96", "CREATE (:A {v: 1}), (:A:B {v: 15}), (:A:C {v: -32}), (:A)",
         Query([Match([NodeP("a", ("A",))])],
               [ret(("list", Collect(P("a", "v")))), Unwind(Var("list"), "item"), ret(("item", Var("item")))]),
         [{"item": 1}, {"item": 15}, {"item": -32}], par),
        ("unwind_list_property", UT + "98-112", "CREATE (:A {v: [1, 2]}), (:A:B {v: [-4]})",
         Query([Match([NodeP("a", ("A",))])],
               [ret(("list", P("a", "v"))), Unwind(Var("list"), "item"), ret(("item", Var("item")))]),
         [{"item": 1}, {"item": 2}, {"item": -4}], dict(par, **lo)),
        ("unwind_null_literal", UT + "134-145", "CREATE (:A)",
         Query([Unwind(NullLit(), "item")], [ret(("item", Var("item")))]), []),
        ("unwind_null_expression", UT + "147-160", "CREATE (:A)",
         Query([Match([NodeP("a", ("A",))])],
               [ret(("list", P("a", "v")), ("a", N("a"))), Unwind(Var("list"), "item"),
                ret(("a", N("a")), ("item", Var("item")))]), []),
        ("unwind_involved", UT + "162-183", chain,
         Query([arb, Unwind(Param("param"), "item")],
               [ret(("a", N("a")), ("r", Var("r", "RELATIONSHIP")), ("item", Var("item")),
                    where=[GreaterThan(Var("item"), IntegerLit(1))]),
                ret(("a", N("a")), ("item", Var("item")))]),
         [{"a": a, "item": i} for a in (na, nb) for i in (2, 3)], par),
    ]


VALS3 = "CREATE (:Node {val: 4}),(:Node {val: 3}),(:Node  {val: 42})"


def _with_cases():
    nm = Match([NodeP("n", ("Node",)), NodeP("m", ("Node",))], [RelP("r", "n", "m")])
    two = "CREATE (:Node {val: 4})-[:Rel]->(:Node {val: 5})"
    val = lambda **kw: Query([Match([NodeP("a")])],  # noqa: E731
                             [ret(("val", P("a", "val")), **kw), ret(("val", Var("val")))])
    return [
        ("with_rebinding", WT + "37-56", "CREATE (:Node {val: 1}), (:Node {val: 2})",
         Query([Match([NodeP("n", ("Node",))])],
               [ret(("foo", P("n", "val"))), ret(("bar", Add(Var("foo"), IntegerLit(2)))),
                ret(("foo", Add(Var("bar"), IntegerLit(2)))), ret(("foo", Var("foo")))]),
         [{"foo": 5}, {"foo": 6}]),
        ("with_constants", WT + "58-76", "CREATE (), ()",
         Query([Match([NodeP("_a")])],
               [ret(("foo", IntegerLit(3))), ret(("bar", Add(Var("foo"), IntegerLit(2)))), ret(("bar", Var("bar")))]),
         [{"bar": 5}, {"bar": 5}]),
        ("with_variables_in_scope", WT + "78-91", two,
         Query([nm], [ret(("n", N("n")), ("m", N("m"))), ret(("n.val", P("n", "val")))]), [{"n.val": 4}]),
        ("with_property", WT + "93-106", two,
         Query([nm], [ret(("n_val", P("n", "val"))), ret(("n_val", Var("n_val")))]), [{"n_val": 4}]),
        ("with_property_filter", WT + "108-122", "CREATE (:Node {val: 3}), (:Node {val: 4}), (:Node {val: 5})",
         Query([Match([NodeP("n", ("Node",))])],
               [ret(("n_val", P("n", "val")), where=[LessThanOrEqual(Var("n_val"), IntegerLit(4))]),
                ret(("n_val", Var("n_val")))]),
         [{"n_val": 3}, {"n_val": 4}]),
        ("with_addition", WT + "124-137", two,
         Query([nm], [ret(("sum_n_m_val", Add(P("n", "val"), P("m", "val")))), ret(("sum_n_m_val", Var("sum_n_m_val")))]),
         [{"sum_n_m_val": 9}]),
        ("with_aliasing", WT + "139-152", two,
         Query([nm], [ret(("sum", Add(P("n", "val"), P("m", "val")))), ret(("sum2", Var("sum"))),
                      ret(("sum2", Var("sum2")))]),
         [{"sum2": 9}]),
        ("with_mixed_expression", WT + "154-169", "CREATE (:Node {val: 4})-[:Rel]->(:Node {val: 5})-[:Rel]->(:Node)",
         Query([nm], [ret(("n_val", P("n", "val")), ("sum_n_m_val", Add(P("n", "val"), P("m", "val")))),
                      ret(("sum_n_m_val", Var("sum_n_m_val")), ("n_val", Var("n_val")))]),
         [{"sum_n_m_val": 9, "n_val": 4}, {"sum_n_m_val": None, "n_val": 5}]),
        ("with_and_predicates", WT + "171-188", "CREATE ({val1: 1, val2: 3, val3: 10}), ({val1: 1, val2: 2, val3: 3})",
         Query([Match([NodeP("n")])],
               [ret(("val1", P("n", "val1")), ("val2", P("n", "val2")), ("val3", P("n", "val3")),
                    where=[Ands(GreaterThanOrEqual(Var("val1"), IntegerLit(1)), GreaterThan(Var("val2"), IntegerLit(2)),
                                GreaterThan(Var("val3"), IntegerLit(5)))]),
                ret(("val1", Var("val1")), ("val2", Var("val2")), ("val3", Var("val3")))]),
         [{"val1": 1, "val2": 3, "val3": 10}]),
        ("with_order_by", WT + "190-202", VALS3, val(order_by=[("val", "asc")]), [{"val": 3}, {"val": 4}, {"val": 42}]),
        ("with_order_by_asc", WT + "204-216", VALS3, val(order_by=[("val", "asc")]),
         [{"val": 3}, {"val": 4}, {"val": 42}]),
        ("with_order_by_desc", WT + "218-230", VALS3, val(order_by=[("val", "desc")]),
         [{"val": 42}, {"val": 4}, {"val": 3}]),
        ("with_skip", WT + "232-239", VALS3, val(skip=2), None, {"row_count": 1}),
        ("with_order_by_skip", WT + "241-252", VALS3, val(order_by=[("val", "asc")], skip=1), [{"val": 4}, {"val": 42}]),
        ("with_order_by_arithmetic_skip", WT + "254-264", VALS3, val(order_by=[("val", "asc")], skip=IntegerLit(2)),
         [{"val": 42}]),
        ("with_limit", WT + "266-273", VALS3, val(limit=1), None, {"row_count": 1}),
        ("with_order_by_limit", WT + "275-285", VALS3, val(order_by=[("val", "asc")], limit=1), [{"val": 3}]),
        ("with_order_by_arithmetic_limit", WT + "287-298", VALS3, val(order_by=[("val", "asc")], limit=IntegerLit(2)),
         [{"val": 3}, {"val": 4}]),
        ("with_order_by_skip_limit", WT + "300-310", VALS3, val(order_by=[("val", "asc")], skip=1, limit=1),
         [{"val": 4}]),
        ("with_not_literal", WT + "314-332", "CREATE ()",
         Query([], [ret(("t", BoolLit(True)), ("f", BoolLit(False))),
                    ret(("nt", Not(BoolLit(True))), ("nf", Not(BoolLit(False)))),
                    ret(("nt", Var("nt")), ("nf", Var("nf")))]),
         [{"nt": False, "nf": True}]),
        ("with_not_expression", WT + "334-352", "CREATE ({id: 1, val: true}), ({id: 2, val: false})",
         Query([Match([NodeP("n")])], [ret(("id", P("n", "id")), ("val2", Not(P("n", "val")))),
                                       ret(("id", Var("id")), ("val2", Var("val2")))]),
         [{"id": 1, "val2": False}, {"id": 2, "val2": True}]),
    ]


def _return_cases():
    aa = "CREATE (:A {name: 'me'}), (:A)"
    ma = Match([NodeP("a", ("A",))])
    nodes = [node(0, ("A",), name="me"), node(1, ("A",))]
    val = lambda **kw: Query([Match([NodeP("a")])], [ret(("val", P("a", "val")), **kw)])  # noqa: E731
    m = MapExpression([("foo", IntegerLit(123)), ("bar", StringLit("456"))])
    return [
        ("return_only_returned", RT + "41-51", aa,
         Query([ma], [ret(("a", N("a")), ("foo", P("a", "name"))), ret(("a", N("a")))]), [{"a": x} for x in nodes]),
        ("return_tricky_alias", RT + "53-62", aa,
         Query([ma], [ret(("a", N("a")), ("foo", N("a"))), ret(("a", N("a")))]), [{"a": x} for x in nodes]),
        ("return_trickier_alias", RT + "64-75", aa,
         Query([ma], [ret(("a", N("a")), ("foo", N("a"))), ret(("b", N("foo")))]), [{"b": x} for x in nodes]),
        ("return_without_dependencies", RT + "77-85", "CREATE (:A)",
         Query([Match([NodeP("a", ("A",)), NodeP("b")])], [ret(("a", N("a")))]), [{"a": node(0, ("A",))}]),
        ("return_single", RT + "87-93", "CREATE ()", Query([], [ret(("1", IntegerLit(1)))]), [{"1": 1}]),
        ("return_several_columns", RT + "95-101", "CREATE (), ()",
         Query([], [ret(("foo", IntegerLit(1)), ("str", StringLit("")))]), [{"foo": 1, "str": ""}]),
        ("order_by_limit", RT + "292-301", VALS3, val(order_by=[("val", "asc")], limit=1), [{"val": 3}],
         {"ordered": True}),
        ("order_by_arithmetic_limit", RT + "303-313", VALS3, val(order_by=[("val", "asc")], limit=IntegerLit(2)),
         [{"val": 3}, {"val": 4}], {"ordered": True}),
        ("order_by_skip_limit", RT + "315-325", VALS3, val(order_by=[("val", "asc")], skip=1, limit=1),
         [{"val": 4}], {"ordered": True}),
        ("return_map", RT + "328-331", "", Query([], [ret(("m", m))]), [{"m": {"foo": 123, "bar": "456"}}]),
        ("return_map_elements", RT + "339-342", "",
         Query([], [ret(("m", m)), ret(("foo", ElementProperty(Var("m", "MAP"), "foo")),
                                       ("bar", ElementProperty(Var("m", "MAP"), "bar")))]),
         [{"foo": 123, "bar": "456"}]),
    ]


def _optional_cases():
    people = """CREATE (p1:Person {name: "Alice"})
                CREATE (p2:Person {name: "Bob"})
                CREATE (p3:Person {name: "Frank"})
                CREATE (p1)-[:KNOWS]->(p2)
                CREATE (p2)-[:KNOWS]->(p3)
                CREATE (p1)<-[:LOVES]-(p3)"""
    return [
        ("optional_null_row", OT + "41-49", "", Query([Match([NodeP("n")], optional=True)], [ret(("n", N("n")))]),
         [{"n": None}]),
        ("optional_empty_scan_graph", OT + "62-71", "",
         Query([Match([NodeP("n")], optional=True)], [ret(("n", N("n")))]), [{"n": None}]),
        ("optional_stacked", OT + "73-91",
         """CREATE (:DoesExist {property: 42})
            CREATE (:DoesExist {property: 43})
            CREATE (:DoesExist {property: 44})""",
         Query([Match([NodeP("f", ("DoesExist",))], optional=True),
                Match([NodeP("n", ("DoesNotExist",))], optional=True)],
               [ret(("a", Collect(P("n", "property"), True)), ("b", Collect(P("f", "property"), True)))]),
         [{"a": [], "b": [42, 43, 44]}]),
        ("optional_incoming", OT + "241-274", people,
         Query([Match([NodeP("p1", ("Person",)), NodeP("p2", ("Person",))], [RelP("e1", "p1", "p2", ("KNOWS",))]),
                Match([NodeP("p1"), NodeP("p3", ("Person",))], [RelP("e2", "p3", "p1", ("LOVES",))], optional=True)],
               [ret(("p1.name", P("p1", "name")), ("p2.name", P("p2", "name")), ("p3.name", P("p3", "name")))]),
         [{"p1.name": "Alice", "p2.name": "Bob", "p3.name": "Frank"},
          {"p1.name": "Bob", "p2.name": "Frank", "p3.name": None}]),
        # the reference encodes ids as Morpheus byte arrays (List(0)); CAPF's are the LONGs
        ("optional_null_ids", OT + "446-468", 'CREATE (p1:Person {name: "Alice"})',
         Query([Match([NodeP("p1", ("Person",))]),
                Match([NodeP("p1"), NodeP("p2")], [RelP("e1", "p1", "p2")], optional=True)],
               [ret(("id(p1)", Id(N("p1"))), ("id(p2)", Id(N("p2"))))]),
         [{"id(p1)": 0, "id(p2)": None}]),
    ]


def _union_cases():
    """UnionTests.scala :39-264 (tabular UNION / UNION ALL; the graph unions
    :266-300 are catalog features)."""
    one = lambda v: Query([], [ret(("one", IntegerLit(v)))])  # noqa: E731
    unw = lambda *xs: Query([Unwind(_ints(*xs), "i")], [ret(("i", Var("i")))])  # noqa: E731
    ab = 'CREATE (a: A {val: "foo"}) CREATE (b: B {bar: "baz"})'
    na, nb = node(0, ("A",), val="foo"), node(1, ("B",), bar="baz")
    rels = ab + " CREATE (a)-[:REL1 {foo: 42}]->(b) CREATE (b)-[:REL2 {bar: true}]->(a)"
    side = lambda v, lab: Query([Match([NodeP(v, (lab,)), NodeP("_t")], [RelP("r", v, "_t")])],  # noqa: E731
                                [ret(("node", N(v)), ("rel", Var("r", "RELATIONSHIP")))])
    pair = lambda x, lx, y, ly: Query([Match([NodeP(x, (lx,)), NodeP(y, (ly,))])],  # noqa: E731
                                      [ret(("node1", N(x)), ("node2", N(y)))])
    nodes_of = lambda v, lab: Query([Match([NodeP(v, (lab,))])], [ret(("node", N(v)))])  # noqa: E731
    return [
        ("union_all_simple", NT + "39-51", "", UnionQuery(one(1), one(2), all=True), [{"one": 1}, {"one": 2}]),
        ("union_all_stacked", NT + "53-71", "",
         UnionQuery(UnionQuery(UnionQuery(one(1), one(2), True), one(2), True), one(3), True),
         [{"one": 1}, {"one": 2}, {"one": 2}, {"one": 3}]),
        ("union_all_unwind", NT + "73-90", "", UnionQuery(unw(1, 2), unw(1, 2, 6), all=True),
         [{"i": 1}, {"i": 2}, {"i": 1}, {"i": 2}, {"i": 6}]),
        ("union_all_nodes", NT + "92-112", ab, UnionQuery(nodes_of("a", "A"), nodes_of("b", "B"), all=True),
         [{"node": na}, {"node": nb}]),
        ("union_all_nodes_rels", NT + "114-136", rels, UnionQuery(side("a", "A"), side("b", "B"), all=True),
         [{"node": na, "rel": CypherRelationship(2, 0, 1, "REL1", (("foo", 42),))},
          {"node": nb, "rel": CypherRelationship(3, 1, 0, "REL2", (("bar", True),))}]),
        ("union_simple", NT + "140-152", "", UnionQuery(one(1), one(2)), [{"one": 1}, {"one": 2}]),
        ("union_duplicates", NT + "154-165", "", UnionQuery(one(1), one(1)), [{"one": 1}]),
        ("union_stacked", NT + "167-184", "", UnionQuery(UnionQuery(UnionQuery(one(1), one(2)), one(2)), one(3)),
         [{"one": 1}, {"one": 2}, {"one": 3}]),
        ("union_unwind", NT + "186-201", "", UnionQuery(unw(1, 2), unw(1, 2, 6)), [{"i": 1}, {"i": 2}, {"i": 6}]),
        ("union_nodes", NT + "203-223", ab, UnionQuery(pair("a", "A", "b", "B"), pair("b", "B", "a", "A")),
         [{"node1": na, "node2": nb}, {"node1": nb, "node2": na}]),
        ("union_duplicate_nodes", NT + "225-243", 'CREATE (a: A {val: "foo"})',
         UnionQuery(nodes_of("a", "A"), nodes_of("a", "A")), [{"node": node(0, ("A",), val="foo")}]),
        ("union_duplicate_rels", NT + "245-264", "CREATE (a) CREATE (a)-[:REL {val: 42}]->(a)",
         UnionQuery(*[Query([Match([NodeP("_s"), NodeP("_t")], [RelP("r", "_s", "_t")])],
                            [ret(("rel", Var("r", "RELATIONSHIP")))])] * 2),
         [{"rel": CypherRelationship(1, 0, 0, "REL", (("val", 42),))}]),
    ]


def _driving_cases():
    """DrivingTableTests.scala :54-137: `cypher(query, drivingTable = records)`
    — the records (age INTEGER, name STRING) are the plan's Start table."""
    from capf_amd.expr import T_INT, T_STRING
    DT = "MTa/DrivingTableTests.scala:"
    drv = [("age", T_INT, [10, 20, 15], None), ("name", T_STRING, ["Alice", "Bob", "Carol"], None)]
    people = ('CREATE (:Person {name: "George", age: 20}) CREATE (:Person {name: "Frank", age: 50}) '
              'CREATE (:Person {name: "Jon", age: 15})')
    pn = [ret(("p.name", P("p", "name")), ("name", Var("name")))]
    want = [{"p.name": "George", "name": "Bob"}, {"p.name": "Jon", "name": "Carol"}]
    by_age = Match([NodeP("p", ("Person",))], [], [Equals(P("p", "age"), Var("age"))])
    return [
        ("driving_return", DT + "54-63", "", Query([], [ret(("age", Var("age")), ("name", Var("name")))], drv),
         [{"age": 10, "name": "Alice"}, {"age": 20, "name": "Bob"}, {"age": 15, "name": "Carol"}]),
        ("driving_unwind", DT + "65-78", "",
         Query([Unwind(_ints(1, 2), "i")], [ret(("i", Var("i")), ("age", Var("age")), ("name", Var("name")))], drv),
         [{"i": i, "age": a, "name": n} for i in (1, 2) for a, n in ((10, "Alice"), (20, "Bob"), (15, "Carol"))]),
        ("driving_filter", DT + "82-99", people, Query([by_age], pn, drv), want),
        ("driving_pattern_properties", DT + "101-117", people, Query([by_age], pn, drv), want),
        ("driving_complex_match", DT + "119-137",
         'CREATE (b:B) CREATE (:Person {name: "George", age: 20})-[:REL]->(b) '
         'CREATE (:Person {name: "Frank", age: 50})-[:REL]->(b) CREATE (:Person {name: "Jon", age: 15})-[:REL]->(b)',
         Query([by_age, Match([NodeP("p"), NodeP("_t")], [RelP("_r", "p", "_t")])], pn, drv), want),
    ]


# AggregationTests.scala holds four-fifths of its cases in the Flink copy too
# (FTt/acceptance/AggregationTests.scala, transcribed in reference_cases.py);
# the morpheus-only ones are temporal (no Flink lowering) and this one
AGG_CASES = [
    ("count_distinct_grouped", "MTa/AggregationTests.scala:258-277",
     'CREATE (a:Start{id: 1}) CREATE (a)-[:REL]->({val: "foo"}) CREATE (a)-[:REL]->({val: "foo"})',
     Query([Match([NodeP("a", ("Start",)), NodeP("b")], [RelP("_r", "a", "b")])],
           [ret(("a.id", P("a", "id")), ("val", Count(P("b", "val"), True)))]),
     [{"a.id": 1, "val": 1}]),
]


CLAUSE_CASES = _match_cases() + _unwind_cases() + _with_cases() + _return_cases() + _optional_cases() + _union_cases() + _driving_cases() + AGG_CASES

# expected exception class name instead of a Bag (MatchTests.scala:380-418:
# a property whose types conflict across label scans)
_CONFLICT = Query([Match([NodeP("n")])], [ret(("foo", P("n", "f")))])
ERROR_CASES = [
    ("match_conflict_int_string", MT + "380-386", "CREATE (:A {f: 1}), (:B {f: 'hi'})", _CONFLICT,
     "IllegalArgumentException"),
    ("match_conflict_float_string", MT + "388-394", "CREATE (:A {f: 1.2}), (:B {f: 'hi'})", _CONFLICT,
     "IllegalArgumentException"),
    ("match_conflict_bool_string", MT + "396-402", "CREATE (:A {f: true}), (:B {f: 'hi'})", _CONFLICT,
     "IllegalArgumentException"),
    ("match_conflict_bool_int", MT + "404-410", "CREATE (:A {f: true}), (:B {f: 1})", _CONFLICT,
     "IllegalArgumentException"),
    ("match_conflict_bool_int_string", MT + "412-418", "CREATE (:A {f: true}), (:B {f: 1}), (:C {f: 'hi'})",
     _CONFLICT, "IllegalArgumentException"),
    ("expr_property_any_type", "MTa/ExpressionTests.scala:342-352", "CREATE (:A {val: 'foo'}), (:B {val: 1}), (:C)",
     Query([Match([NodeP("a")])], [ret(("a.val", P("a", "val")))]), "IllegalArgumentException"),
]
