"""Headline benchmark: 2-hop MATCH count(*) on R-MAT scale 24 (BASELINE.json).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--scale 24]

One step = one execution of
    MATCH (a)-->(b)-->(c) RETURN count(*)
planned through the okapi relational lowering (planner.py → Table SPI →
libcapf_gpu.so) over the HBM-resident R-MAT graph: plan build, fused
factorised count on the GPU, scalar result back on the host.  The graph is
generated on the device before the timed region (inputs resident in HBM).

value = joined rows/s = count(*) (path multiplicity) / median step time, whole
job: the K timed steps are K single queries, each from the plan call to the
scalar on the host; the pipelined serving rate is a side field.
For N > 1 the graph is hash-partitioned over one process per GPU (dist.py);
ranks are launched by torch.distributed.run, and the max over ranks is timed.
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import capf_import  # noqa: E402,F401

METRIC = "joined rows/sec for 2-hop MATCH on R-MAT s24 at 1/2/4/8 GPUs; % HBM roofline"
ROWS_METRIC = "joined rows/sec for MATCH (a)-->(b) RETURN a, b materialised on R-MAT (materialising join leg)"
ONE_HOP_METRIC = "joined rows/sec for 1-hop MATCH (a:Person)-->(b) count(*) on R-MAT (config 2)"
TRI_METRIC = "joined rows/sec for triangle MATCH (a)-->(b)-->(c)-->(a) on R-MAT (config 4)"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def two_hop_query():
    from capf_amd.expr import CountStar
    from capf_amd.planner import Match, NodeP, Query, RelP, Stage
    return Query([Match([NodeP("a"), NodeP("b"), NodeP("c")], [RelP("r1", "a", "b"), RelP("r2", "b", "c")])],
                 [Stage([("count", CountStar())])])


def triangle_query():
    from capf_amd.expr import CountStar
    from capf_amd.planner import Match, NodeP, Query, RelP, Stage
    return Query([Match([NodeP("a"), NodeP("b"), NodeP("c")],
                        [RelP("r1", "a", "b"), RelP("r2", "b", "c"), RelP("r3", "c", "a")])],
                 [Stage([("count", CountStar())])])


def one_hop_person_query():
    from capf_amd.expr import CountStar
    from capf_amd.planner import Match, NodeP, Query, RelP, Stage
    return Query([Match([NodeP("a", ("Person",)), NodeP("b")], [RelP("r", "a", "b")])],
                 [Stage([("count", CountStar())])])


def one_hop_rows_query():
    """MATCH (a)-->(b) RETURN a, b — the materialising Expand join (2 joins
    of RelationalPlanner.scala:130-165 through the materialising joins)."""
    from capf_amd.expr import Var
    from capf_amd.planner import Match, NodeP, Query, RelP, Stage
    return Query([Match([NodeP("a"), NodeP("b")], [RelP("r", "a", "b")])],
                 [Stage([("a", Var("a", "NODE")), ("b", Var("b", "NODE"))])])


def var2_rows_query():
    """MATCH (a)-[*2..2]->(b) RETURN a, b — the relational VarLengthExpand
    (VarLengthExpandPlanner.scala:82-135): the path step joins end(r_1) =
    start(r_2), a many-to-many join of two rel scans (no unique side: the
    radix-partitioned join's case), then the uniqueness filter r_1 <> r_2 and
    the target join."""
    from capf_amd.expr import Var
    from capf_amd.planner import Match, NodeP, Query, RelP, Stage
    return Query([Match([NodeP("a"), NodeP("b")], [RelP("r", "a", "b", length=(2, 2))])],
                 [Stage([("a", Var("a", "NODE")), ("b", Var("b", "NODE"))])])


def reach_query(upper=3):
    """Config 5: MATCH (a:Person)-[:KNOWS*1..3]->(b:Person) WITH DISTINCT a, b
    WITH a, count(*) AS reach RETURN reach, count(*) AS n."""
    from capf_amd.expr import CountStar, Var
    from capf_amd.planner import Match, NodeP, Query, RelP, Stage
    return Query([Match([NodeP("a", ("Person",)), NodeP("b", ("Person",))],
                        [RelP("k", "a", "b", ("KNOWS",), length=(1, upper))])],
                 [Stage([("a", Var("a")), ("b", Var("b"))], distinct=True),
                  Stage([("a", Var("a")), ("reach", CountStar())]),
                  Stage([("reach", Var("reach")), ("n", CountStar())])])


def workload_name(args):
    if args.query == "var2_rows":
        return f"R-MAT s{args.scale} MATCH (a)-[*2..2]->(b) RETURN a, b (relational var-length, rows in HBM)"
    if args.query == "one_hop_rows":
        return (f"R-MAT s{args.scale} 1-hop MATCH (a)-->(b) RETURN a, b (rows materialised in HBM)"
                + (f", sparse node ids v*{args.id_stride}+7" if args.id_stride != 1 else ""))
    if args.query == "one_hop_person":
        return f"R-MAT s{args.scale} 1-hop MATCH (a:Person)-->(b) RETURN count(*)"
    if args.query == "triangle":
        return f"R-MAT s{args.scale} triangle MATCH (a)-->(b)-->(c)-->(a) RETURN count(*)"
    if args.query == "reach":
        return (f"config 5: LDBC-SF10-shaped KNOWS (2^{args.scale} Person, R-MAT edge factor {args.edge_factor}) "
                f"MATCH (a:Person)-[:KNOWS*1..3]->(b:Person) WITH DISTINCT a, b WITH a, count(*) AS reach "
                f"RETURN reach, count(*) AS n")
    return f"R-MAT s{args.scale} 2-hop MATCH (a)-->(b)-->(c) RETURN count(*)"


CPU_THREAD_CAP = 16  # the GPU box's CPU share for one GPU (OMP_NUM_THREADS there)


def cpu_available():
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def cpu_threads():
    return max(1, min(CPU_THREAD_CAP, cpu_available()))


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def cpu_info(threads):
    """The host the CPU baseline ran on: model, cores visible, threads used, cap."""
    return {"cpu_model": cpu_model(), "host_cores_visible": cpu_available(), "threads_used": threads,
            "thread_cap": CPU_THREAD_CAP,
            "cap_reason": "one GPU's share of the box's CPUs (OMP_NUM_THREADS=16 on the GPU box)"}


def tri_cpu_baseline(session, graph, scale, budget_s):
    """Config 4 on the host cores, Flink plan shape (oracle/rmat.c
    pipeline_triangles): hash tables on the full node scan, the start-keyed R2
    and the (start, end)-keyed R3 (built, not timed), then the first K r1 rows
    expand through R2 — every wedge row materialised — and probe R3 on both
    keys with the three uniqueness filters (RelationalPlanner.scala:130-189).
    value = triangle rows / probe seconds over that bounded sample."""
    import numpy as np
    from oracle import cmodel
    rel = graph.rel_tables[0].table
    src, _ = rel.column_arrays("source")
    dst, _ = rel.column_arrays("target")
    ids, _ = rel.column_arrays("id")
    nodes = np.arange(1 << scale, dtype=np.int64)
    th = cpu_threads()
    t0 = time.perf_counter()
    pipe = cmodel.Pipeline(nodes, ids, src, dst, threads=th)
    pipe.build_pairs(th)
    build_s = time.perf_counter() - t0
    m = len(src)
    k = min(m, 1 << 12)
    tris, wedges, probe_s, lo = 0, 0, 0.0, 0
    while lo < m:  # grow the sample until the probe budget is used
        hi = min(m, lo + k)
        t0 = time.perf_counter()
        c, w = pipe.triangles(lo, hi, th)
        probe_s += time.perf_counter() - t0
        tris, wedges, lo = tris + c, wedges + w, hi
        if probe_s >= budget_s:
            break
        k *= 2
    pipe.close()
    return {"value": tris / probe_s if probe_s > 0 else None, "unit": "joined rows/s", "cores": th,
            **cpu_info(th), "kind": "port",
            "sample": (f"R-MAT s{scale} triangle, Flink plan shape (hash tables on the node scan, start-keyed R2 "
                       f"and (start, end)-keyed R3, {build_s:.1f}s build, not timed); r1 rows [0,{lo}) of {m}: "
                       f"{wedges} wedge rows probed, {tris} triangle rows in {probe_s:.2f}s on {th} threads")}


def c2_cpu_baseline(graph, scale):
    """Config 2 on the host cores: the Flink plan shape (oracle/rmat.c
    onehop_label_count) — hash-join builds on the Person scan and the all-node
    scan, then every rel through both probes, counted — on the box's threads
    (capped at one GPU's share); the whole workload, builds included (Flink
    builds its hash tables per query), no sample needed."""
    import numpy as np
    from oracle import cmodel
    rel = graph.rel_tables[0].table
    src, _ = rel.column_arrays("source")
    dst, _ = rel.column_arrays("target")
    pid, _ = graph.node_tables[0].table.column_arrays("id")
    oid, _ = graph.node_tables[1].table.column_arrays("id")
    allid = np.concatenate([np.asarray(pid, dtype=np.int64), np.asarray(oid, dtype=np.int64)])
    th = cpu_threads()
    t0 = time.perf_counter()
    count = cmodel.onehop_label_count(pid, allid, src, dst, threads=th)
    el = time.perf_counter() - t0
    return {"value": count / el, "unit": "joined rows/s", "cores": th, **cpu_info(th), "kind": "port",
            "count": count,
            "sample": (f"whole R-MAT s{scale} workload ({len(src)} rels): (a:Person)-->(b), Flink plan shape "
                       f"(hash-join builds on both node scans + probes, oracle/rmat.c onehop_label_count) in "
                       f"{el:.3f}s on {th} threads")}


def cpu_baseline(session, graph, scale, budget_s):
    """Flink-shaped pipelined hash join (oracle/rmat.c) on the host cores over
    a bounded sample of the same workload: hash tables are built on the full
    node scan and the full R2 (start-keyed); the first K r1 rows probe them."""
    import numpy as np
    from oracle import cmodel
    rel = graph.rel_tables[0].table
    src, _ = rel.column_arrays("source")
    dst, _ = rel.column_arrays("target")
    ids, _ = rel.column_arrays("id")
    nodes = np.arange(1 << scale, dtype=np.int64)
    th = cpu_threads()
    t0 = time.perf_counter()
    pipe = cmodel.Pipeline(nodes, ids, src, dst, threads=th)
    build_s = time.perf_counter() - t0
    m = len(src)
    k = min(m, 1 << 16)
    rows, probe_s = 0, 0.0
    lo = 0
    while lo < m:  # grow the sample until the probe budget is used
        hi = min(m, lo + k)
        t0 = time.perf_counter()
        rows += pipe.probe(lo, hi, th)
        probe_s += time.perf_counter() - t0
        lo = hi
        if probe_s >= budget_s:
            break
        k *= 2
    pipe.close()
    return {
        "value": rows / probe_s if probe_s > 0 else None,
        "unit": "joined rows/s",
        "cores": th,
        **cpu_info(th),
        "kind": "port",
        "sample": (f"R-MAT s{scale} 2-hop, Flink plan shape (hash tables on the full node scan and "
                   f"start-keyed R2, {build_s:.1f}s build, not timed); probe of r1 rows [0,{lo}) of {m} "
                   f"producing {rows} joined rows in {probe_s:.2f}s on {th} threads"),
    }


# kernels of one fused 2-hop count (fused_count.hip + chain2_partitioned.hip)
PIPELINE = ("c5_partition", "c3_transpose", "c3_units", "c3_zero", "c5_gather", "c3_overflow", "chain2_hist", "message_pass",
            "semi_partition", "semi_count",
            "chain2_dot", "tri_keys", "tri_sort_keys", "tri_rle", "tri_pairs", "tri_orient",
            "tri_sort_pairs", "tri_rowptr", "tri_split", "tri_loop3", "tri_count", "tri_count_packed",
            "tri_count_qtiled", "tri_count_passb",
            "rj_partition1", "rj_partition2", "rj_join_count", "rj_join_emit", "gather")

# kernel symbols behind a timer label (the default is "k_" + label); PMC files are
# matched against these, template arguments stripped
PMC_SYMBOLS = {"chain2_dot": ("k_chain2_dot", "k_chain2_dot_pairs"),
               "semi_partition": ("k_c5_shard_partition",), "semi_count": ("k_c5_bits_count",)}


def lib_digest():
    """sha256 prefix of the loaded libcapf_gpu.so (matched against the PMC
    file's `lib`: the traffic figure must describe the benched build)."""
    import hashlib
    from capf_amd import _lib
    with open(_lib.LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def pmc_symbols(label):
    return PMC_SYMBOLS.get(label, ("k_" + label,))


def load_pmc(path, labels):
    """A committed PMC summary (tools/make_pmc_json.py) — only when its kernels
    are the kernels that ran: every timer label in `labels` (profiled pass) must
    have one of its kernel symbols in the file, else the file describes another
    build's kernels and is refused.  Returns (json or None, provenance dict)."""
    rel = os.path.relpath(path, ROOT)
    if not os.path.exists(path):
        return None, {"file": rel, "rejected": "not collected"}
    with open(path) as f:
        j = json.load(f)
    names = {k.split("<")[0].strip() for k in j.get("kernels", {})}
    missing = [lb for lb in labels if not any(sym in names for sym in pmc_symbols(lb))]
    prov = {"file": rel, "lib": j.get("lib"), "pmc_kernels": sorted(j.get("kernels", {})),
            # which kernel symbols each timer label of the line stands for
            "timer_kernels": {lb: list(pmc_symbols(lb)) for lb in labels}}
    if missing:
        prov["rejected"] = f"no counters for kernels that ran: {missing}"
        return None, prov
    return j, prov


def pmc_bytes_of(j, labels):
    """Corrected HBM bytes per launch of the kernels behind `labels`."""
    syms = {sym for lb in labels for sym in pmc_symbols(lb)}
    return sum(v["read_bytes"] + v["write_bytes"] for k, v in j["kernels"].items()
               if k.split("<")[0].strip() in syms)


def pipeline_roofline(prof, steps, compulsory_bytes, traffic_per_query=None):
    """Roofline of the fused count as one unit: the compulsory bytes of the
    query (src+dst at int64 width + node ids) over the summed
    device time of its kernels per query, measured with HIP events on the
    session stream.  The per-kernel split is reported beside it."""
    per = {k: v["total_ms"] / steps for k, v in prof.items() if k in PIPELINE}
    kern_ms = sum(per.values())
    achieved = compulsory_bytes / (kern_ms * 1e-3) / 1e9 if kern_ms > 0 else None
    dom = max(per, key=per.get) if per else None
    return {
        "bound": "hbm",
        "kernel": "fused 2-hop count pipeline (" + " + ".join(sorted(per)) + ")",
        "achieved": achieved,
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
        "traffic": traffic_per_query,
        "algorithmic_bytes_per_launch": compulsory_bytes,
        "pipeline_ms_per_query": kern_ms,
        "kernel_ms_per_query": per,
        "dominant_kernel": dom,
    }


def tri_roofline(prof, steps, n_nodes, traffic_per_query=None):
    """Config 4: compulsory bytes are not meaningful — the work
    is closing-edge probes.  Roofline of the dominant kernel tri_count over ITS
    algorithmic bytes: 4 B per probe (the neighbour id w of N+(q), searched in
    the LDS copy of N+(p)), 16 B per hit (the two multiplicity pairs), 20 B per
    oriented edge (rowptr pair, multiplicity pair, staged column) and 8 B per
    node row; probe / hit / edge counts come from the kernel's own counters
    (profiled pass).  `traffic` = PMC bytes of tri_count (rocprofv3 FETCH×2 +
    WRITE, profiles/pmc_tri_s<scale>.json) when collected."""
    per = {k: v["total_ms"] / steps for k, v in prof.items() if k in PIPELINE}
    probes = prof.get("tri_probes", {}).get("bytes", 0.0) / steps
    hits = prof.get("tri_hits", {}).get("bytes", 0.0) / steps
    probes_a = prof.get("tri_probes_pass_a", {}).get("bytes", 0.0) / steps
    edges = prof.get("tri_oriented_edges", {}).get("bytes", 0.0) / steps
    labs = [k for k in per if k.startswith("tri_count")]  # pass A (row by row or q-tiled) + pass B
    lab = " + ".join(sorted(labs)) or "tri_count"
    t = sum(per[k] for k in labs)
    algo = 4.0 * probes + 16.0 * hits + 20.0 * edges + 8.0 * n_nodes
    achieved = algo / (t * 1e-3) / 1e9 if t > 0 else None
    return {
        "bound": "hbm", "kernel": f"{lab} (closing-edge probes)",
        "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": achieved / HBM_PEAK_GBS if achieved else None,
        "traffic": traffic_per_query, "algorithmic_bytes_per_launch": algo,
        "probes_per_launch": probes, "hits_per_launch": hits, "oriented_edges": edges,
        "probes_pass_a": probes_a, "probes_pass_b": probes - probes_a,
        "passb_edges": prof.get("tri_passb_edges", {}).get("bytes", 0.0) / steps,
        "passa_items": prof.get("tri_passa_items", {}).get("bytes", 0.0) / steps,
        "probes_per_s": probes / (t * 1e-3) if t > 0 else None,
        "kernel_ms": t, "pipeline_ms_per_query": sum(per.values()), "kernel_ms_per_query": per,
        "note": "compulsory 16·M + 8·N bytes are not meaningful for config 4 (SURVEY §8(d)); "
                "value is rows/s, the roofline is the count kernel's probe traffic",
    }


def id_width(args):
    """Ingest-time id encoding of the synthetic graph: False = plain int64,
    4 = FOR32, 3 = FOR24 (3-byte offsets + base where the range fits 24 bits,
    FOR32 otherwise).  The values are the reference's int64 ids either way."""
    if args.int64:
        return False
    return 3 if args.query in ("two_hop", "one_hop_person") and not args.for32 else 4


def id_storage(args):
    return {False: "int64", 4: "FOR32 (uint32 offsets + base; int64 values)",
            3: "FOR24 (3-byte offsets + base where the range fits 24 bits; int64 values)"}[id_width(args)]


def timed_singles(fn, steps, sync):
    """K single steps, each bracketed by a device sync; (last result, seconds per step)."""
    out, times = None, []
    for _ in range(steps):
        sync()
        t0 = time.perf_counter()
        out = fn()
        times.append(time.perf_counter() - t0)
    sync()
    return out, times


def timed_steps(fn, steps, sync):
    sync()
    t0 = time.perf_counter()
    out = None
    for _ in range(steps):
        out = fn()
    sync()
    return out, time.perf_counter() - t0


def run_rows_leg(args):
    """Materialising join leg: K steps of plan + evaluation of
    MATCH (a)-->(b) RETURN a, b into device memory (no download), ids FOR32.
    Compulsory bytes (SURVEY §8(d) style): src+dst at int64 width (16 B/rel),
    the two node scans (8 B/node each) and the result (a, b: 16 B/row + the
    1-B label flag of each node)."""
    from capf_amd.planner import plan_query
    from capf_amd.synthetic import rmat_graph
    from capf_amd.table import GpuSession
    s = GpuSession(0)
    g = rmat_graph(s, args.scale, args.edge_factor, compact=True, id_stride=args.id_stride)
    var2 = args.query == "var2_rows"
    q = var2_rows_query() if var2 else one_hop_rows_query()
    n_nodes = 1 << args.scale
    m = args.edge_factor << args.scale
    step = lambda: plan_query(g, q).table.materialize()  # noqa: E731
    rows = plan_query(g, q).table.size
    if var2:  # one row per 2-path with distinct rels: the 2-hop count fixture
        want = fixture_count("two_hop", args.scale, args.edge_factor)
        if want is not None and rows != want:
            raise SystemExit(f"{rows} rows, expected the 2-hop fixture {want}")
    elif rows != m:
        raise SystemExit(f"{rows} rows, expected one per rel ({m})")
    for _ in range(args.warmup):
        step()
    s.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    s.sync()
    elapsed = time.perf_counter() - t0
    s.reset_profile()
    s.set_profiling(True)
    prof_steps = max(1, min(args.steps, 5))
    for _ in range(prof_steps):
        step()
    s.sync()
    s.set_profiling(False)
    prof = s.profile()
    per = {k: v["total_ms"] / prof_steps for k, v in prof.items()}
    kern_ms = sum(per.values())
    # var2: both rel scans are read (the path step and its start/target joins)
    compulsory = (32.0 if var2 else 16.0) * m + 16.0 * n_nodes + 18.0 * rows
    ms = elapsed * 1e3 / args.steps
    # the sparse-id leg's HBM bytes per step: the PMC passes of
    # tools/collect_rows_pmc.sh over its hashed-index probes (the step's
    # dominant kernel, two launches per step), when collected for this build
    traffic, tsrc = None, None
    if not var2 and args.id_stride != 1 and per.get("hidx_probe"):
        j, tsrc = load_pmc(os.path.join(ROOT, "profiles", f"pmc_rows_sparse_s{args.scale}.json"), ["hidx_probe"])
        if j is not None and tsrc.get("lib") == "libcapf_gpu.so sha256:" + lib_digest():
            launches = prof.get("hidx_probe", {}).get("launches", 2 * prof_steps) / prof_steps
            traffic = pmc_bytes_of(j, ["hidx_probe"]) * launches
        elif j is not None:
            tsrc["rejected"] = "collected for another build"
    print(json.dumps({
        "metric": ROWS_METRIC, "value": rows * args.steps / elapsed, "unit": "joined rows/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms, "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "int64",
        "data": f"synthetic R-MAT s{args.scale} generated in HBM before timing",
        "config": {"workload": workload_name(args), "scale": args.scale, "nodes": n_nodes, "rels": m,
                   "rows": rows, "id_storage": "FOR32" if args.id_stride == 1 else
                   f"int64, sparse ids v*{args.id_stride}+7 (no FOR: the range exceeds 32 bits)",
                   "plan": s.last_plan() or "relational (2 joins)",
                   "join": {"radix": "radix-partitioned (csrc/radix_join.hip), forced by CAPF_JOIN=radix",
                            "hash": "global hash table (csrc/kernels_hash.hip), forced by CAPF_JOIN=hash"}.get(
                       os.environ.get("CAPF_JOIN", ""),
                       "planner choice: direct-address join on the dense node-id key, hashed unique-key index "
                       "on sparse node ids (csrc/dense_join.hip), radix-partitioned join (csrc/radix_join.hip) "
                       "for non-unique keys")},
        # the step runs many small kernels (two joins, gathers, scans): the
        # roofline is taken over the whole step's wall time; the timed
        # kernels' split (partition / join passes) is reported beside it
        "roofline": ({"bound": "hbm", "kernel": "whole step (2 joins + gathers + scans), wall time",
                      "achieved": compulsory / (ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                      "frac": compulsory / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                      "traffic": traffic, "traffic_scope": "hidx_probe launches of one step" if traffic else None,
                      "traffic_source": tsrc, "algorithmic_bytes_per_launch": compulsory,
                      "timed_kernels_ms_per_step": per, "timed_kernels_ms_sum": kern_ms}
                     if kern_ms > 0 else
                     {"bound": "hbm", "kernel": "none: no kernel ran — the result's (a, b) columns ARE the rel "
                      "table's source / target columns (both node scans hold only their ids and every endpoint "
                      "lies in the dense id range by the cached statistics, so both Expand joins are identities "
                      "on the rel rows: zero-copy, csrc/dense_join.hip)",
                      "achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": None, "traffic": None,
                      "algorithmic_bytes_per_launch": compulsory, "timed_kernels_ms_per_step": per,
                      "timed_kernels_ms_sum": kern_ms}),
    }))


REACH_METRIC = ("distinct (a, b) pairs/sec for config 5: [:KNOWS*1..3] var-length expand + DISTINCT + "
                "GROUP BY on an LDBC-SF10-shaped graph")


def reach_cpu_baseline(src, dst, n, budget_s):
    """The relational plan's shape on the host cores (oracle/rmat.c::reach_paths):
    per sampled source every isomorphic path of 1..3 rels (the join chain with
    the isomorphism filters, VarLengthExpandPlanner.scala:82-259), end nodes
    deduplicated (DISTINCT a, b) and counted (GROUP BY a).  The sample grows
    until the budget is used; value = distinct pairs found / second."""
    import numpy as np
    from oracle import cmodel
    th = cpu_threads()
    rng = np.random.default_rng(5)
    order = rng.permutation(n)
    k, lo, pairs, paths, secs = 64, 0, 0, 0, 0.0
    while lo < n and secs < budget_s:
        part = np.sort(order[lo:lo + k])
        t0 = time.perf_counter()
        r, p = cmodel.reach_paths(src, dst, n, part, 3, th)
        secs += time.perf_counter() - t0
        pairs += int(r.sum())
        paths += p
        lo += k
        k *= 2
    return {"value": pairs / secs if secs > 0 else None, "unit": "distinct (a, b) pairs/s", "cores": th,
            **cpu_info(th), "kind": "port",
            "sample": (f"config 5 relational plan shape (isomorphic paths of 1..3 rels per source, DISTINCT, "
                       f"GROUP BY) for {lo} of {n} random sources: {paths} paths, {pairs} distinct pairs "
                       f"in {secs:.2f}s on {th} threads")}


def run_reach_leg(args):
    """Config 5 at its BASELINE size: 2^16 Person nodes, R-MAT
    KNOWS rels with edge factor 30, MATCH (a:Person)-[:KNOWS*1..3]->(b:Person)
    WITH DISTINCT a, b WITH a, count(*) AS reach RETURN reach, count(*) AS n
    through the planner: the unchanged relational plan (join chains, UNION ALL,
    DISTINCT, GROUP BY) whose Group the runtime recognises in its plan DAG and
    evaluates by the fused var-length reach (fused_count.hip::try_fused_reach →
    csrc/var_length_reach.hip).  A step = plan call → the histogram rows on the host; value = distinct (a, b)
    pairs / median step.  Parity: the histogram is the committed fixture
    (tests/golden/config5_sf10.json, C bitset BFS)."""
    import torch  # noqa: F401
    from capf_amd.graph import ElementTable, ScanGraph
    from capf_amd.planner import run
    from capf_amd.synthetic import rmat_seed, thresholds
    from capf_amd.table import GpuSession
    s = GpuSession(0)
    m = args.edge_factor << args.scale
    n = 1 << args.scale
    rels = s.rmat_rels(args.scale, rmat_seed(args.scale), thresholds(), 0, m)
    nodes = s.range_nodes(0, n, id_col="id")
    g = ScanGraph(s, [ElementTable("node", frozenset(["Person"]), nodes, {})],
                  [ElementTable("rel", frozenset(["KNOWS"]), rels, {})])
    q = reach_query()
    step = lambda: run(g, q)  # noqa: E731
    t0 = time.perf_counter()
    s.reset_profile()
    res = step()
    first_ms = (time.perf_counter() - t0) * 1e3
    if s.last_plan() != "fused_var_length_reach":
        raise SystemExit(f"config 5 did not take the fused reach (plan {s.last_plan()})")
    for _ in range(args.warmup):
        step()
    res, times = timed_singles(step, args.steps, s.sync)
    hist = sorted([r["reach"], r["n"]] for r in res)
    pairs = sum(r * c for r, c in hist)
    median_ms = statistics.median(times) * 1e3
    parity = {"fixture": None, "match": False}
    fx = os.path.join(ROOT, "tests", "golden", "config5_sf10.json")
    if os.path.exists(fx) and (args.scale, args.edge_factor) == (16, 30):
        with open(fx) as f:
            want = json.load(f)["histogram"]
        if hist != want:
            raise SystemExit("config 5 histogram differs from the committed fixture")
        parity = {"fixture": "tests/golden/config5_sf10.json", "match": True, "histogram_rows": len(want)}
    s.reset_profile()
    s.set_profiling(True)
    prof_steps = max(1, min(args.steps, 5))
    for _ in range(prof_steps):
        step()
    s.sync()
    s.set_profiling(False)
    prof = s.profile()
    per = {k: v["total_ms"] / prof_steps for k, v in prof.items()}
    lev = prof.get("vr_level", {})
    lev_ms = lev.get("total_ms", 0.0) / max(1, lev.get("launches", 1))
    lev_bytes = lev.get("bytes", 0.0) / max(1, lev.get("launches", 1))  # nominal frontier traffic
    j, pmc_prov = load_pmc(os.path.join(ROOT, "profiles", f"pmc_reach_s{args.scale}.json"), ["vr_level"])
    traffic = pmc_bytes_of(j, ["vr_level"]) if j is not None else None  # per vr_level dispatch
    # the roofline is taken on the bytes the counters saw (FETCH x2 + WRITE per
    # vr_level launch): the nominal frontier figure counts every in-edge's word
    # pull, most of which the Infinity Cache serves
    achieved = traffic / (lev_ms * 1e-3) / 1e9 if traffic and lev_ms > 0 else None
    # the bytes of materialised intermediates per query =
    # the HBM bytes the query's kernels WRITE (PMC WRITE_SIZE), per-dispatch values
    # times dispatches per query (the PMC run's query count = k_vr_count_bs's)
    inter = None
    if j is not None:
        ks = j["kernels"]
        nq = max(1, ks.get("k_vr_count_bs", {}).get("dispatches", 1))
        inter = sum(v["write_bytes"] * (v["dispatches"] / nq) for k, v in ks.items()
                    if v["dispatches"] >= nq)  # per-query kernels (the cached index is built once)
    result = {
        "metric": REACH_METRIC, "value": pairs / (median_ms * 1e-3), "unit": "distinct (a, b) pairs/s",
        "n_gpus": 1, "steps": args.steps, "warmup": args.warmup, "ms_per_step": median_ms,
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "int64",
        "data": (f"synthetic LDBC-SF10-shaped graph: R-MAT s{args.scale} (Graph500 a/b/c), edge factor "
                 f"{args.edge_factor}, every node a Person, generated in HBM before timing"),
        "config": {"workload": workload_name(args), "scale": args.scale, "nodes": n, "rels": m,
                   "distinct_pairs": pairs, "sources_reaching": sum(c for _, c in hist),
                   "plan": ("relational plan through the Table SPI; Group(a; count) over Distinct(a, b) over the "
                            "UNION ALL of the *1..3 join chains recognised in the runtime DAG → fused "
                            "var-length reach (try_fused_reach)"),
                   "steps_mode": "K single queries, plan call -> histogram rows on the host; value = pairs / median",
                   "ms_per_query_mean": sum(times) * 1e3 / len(times), "ms_per_query_min": min(times) * 1e3,
                   "first_query_ms": first_ms, "parity": parity},
        "roofline": {
            "bound": "hbm", "kernel": "vr_level (pull BFS level, 64 sources per uint64 word)",
            "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS if achieved else None, "traffic": traffic,
            "achieved_basis": "PMC HBM bytes per vr_level launch (traffic) / its HIP-event time; null without "
                              "a PMC summary of this build's kernels",
            "nominal_bytes_per_launch": lev_bytes,
            "nominal_bytes_definition": ("8 B per rel per source word (the source's frontier word, pulled "
                                         "along every in-edge) + 24 B per node per source word (frontier, "
                                         "next frontier, visited); mostly Infinity-Cache hits"),
            "materialized_intermediate_bytes_per_query": inter,
            "materialized_intermediate_definition": ("PMC WRITE_SIZE of the per-query vr_* kernels (BFS "
                                                     "frontier / visited words, counts); the relational plan "
                                                     "would materialise every path row (≈1e10 x 40 B)"),
            "kernel_ms": lev_ms, "kernel_ms_per_query": per, "device_ms_per_query": sum(per.values()),
            "traffic_source": pmc_prov},
    }
    if not args.no_cpu:
        src, _ = rels.column_arrays("source")
        dst, _ = rels.column_arrays("target")
        result["cpu_baseline"] = reach_cpu_baseline(src, dst, n, args.cpu_seconds)
    print(json.dumps(result))


def run_single(args):
    import torch  # noqa: F401  (HIP runtime, device selection)
    from capf_amd.planner import run
    from capf_amd.synthetic import rmat_graph
    from capf_amd.table import GpuSession

    s = GpuSession(0)
    g = rmat_graph(s, args.scale, args.edge_factor, compact=id_width(args),
                   person_split=args.query == "one_hop_person")
    q = {"triangle": triangle_query, "one_hop_person": one_hop_person_query}.get(args.query, two_hop_query)()
    n_nodes = 1 << args.scale
    m = args.edge_factor << args.scale
    step = lambda: run(g, q)[0]["count"]  # noqa: E731
    # the first query also builds what is cached per graph (scan unions, column
    # statistics, the triangle's oriented CSR): reported, never timed as a step
    t_first = time.perf_counter()
    step()
    first_query_ms = (time.perf_counter() - t_first) * 1e3
    for _ in range(args.warmup):
        step()
    # SURVEY §8(d) / BASELINE.md: the K timed steps are K single queries, each
    # plan call → scalar result on the host, bracketed by a device sync; value
    # and ms_per_step come from their MEDIAN
    count, times = timed_singles(step, args.steps, s.sync)
    median_ms = statistics.median(times) * 1e3
    pipelined_ms = None
    if not args.sync_steps and args.query != "triangle":
        # side figure (not the value): pipelined serving — step i plans query i
        # on the host and enqueues its fused count into slot i
        # (capf_table_count_async) while the GPU still runs query i−1; every
        # query is planned and counted in full, the K counts are downloaded and
        # checked after the closing synchronize
        import torch
        from capf_amd.planner import plan_query
        slots = torch.zeros(args.steps, dtype=torch.int64, device="cuda")
        base = slots.data_ptr()
        torch.cuda.synchronize()  # zero-fill on torch's stream, counts on the session stream

        def enqueue(i):
            plan_query(g, q).table.count_async(base + 8 * i)

        for i in range(min(args.warmup, args.steps)):
            enqueue(i)
        s.sync()
        t0 = time.perf_counter()
        for i in range(args.steps):
            enqueue(i)
        s.sync()
        pipelined_ms = (time.perf_counter() - t0) * 1e3 / args.steps
        got = slots.cpu().tolist()
        if any(c != count for c in got):
            raise SystemExit(f"pipelined counts {got} differ from the synchronous count {count}")
    # a second, profiled pass attributes the device time to the kernels
    s.reset_profile()
    s.set_profiling(True)
    prof_steps = max(1, min(args.steps, 5))
    timed_steps(step, prof_steps, s.sync)
    s.set_profiling(False)
    prof = s.profile()
    plan = s.last_plan()
    # src+dst at int64 width + node ids (+ the 1-B label for config 2)
    compulsory = 16.0 * m + (9.0 if args.query == "one_hop_person" else 8.0) * n_nodes
    traffic = None
    pfx = {"triangle": "tri_", "one_hop_person": "c2_"}.get(args.query, "")
    pmc = os.path.join(ROOT, "profiles", f"pmc_{pfx}s{args.scale}.json")
    ran = sorted(k for k, v in prof.items() if k in PIPELINE and v["total_ms"] > 0)
    if args.query == "triangle":  # the count kernels (the CSR is built by the first query)
        ran = [k for k in ran if k.startswith("tri_count")]
    j, pmc_prov = load_pmc(pmc, ran)
    if j is not None:
        traffic = pmc_bytes_of(j, ran) if args.query == "triangle" else j.get("hbm_bytes_per_query")
    ms_per_step = median_ms
    if args.query == "triangle":
        roof = tri_roofline(prof, prof_steps, n_nodes, traffic)
    else:
        roof = pipeline_roofline(prof, prof_steps, compulsory, traffic)
        # `achieved` / `frac` on the basis the driver's clock and
        # rocprof reproduce — the compulsory bytes over the median plan -> scalar
        # step (host planning included, so it is the conservative figure); the
        # HIP-event kernel sum of the profiled pass is kept beside it (events
        # between the kernels move P1's dirty-line write-back out of the timed
        # spans, so that sum reads ~5 % below the rocprof kernel-trace sum)
        roof["kernel_event_achieved"] = roof["achieved"]
        roof["kernel_event_frac"] = roof["frac"]
        roof["achieved"] = compulsory / (ms_per_step * 1e-3) / 1e9
        roof["frac"] = roof["achieved"] / HBM_PEAK_GBS
        roof["basis"] = "compulsory bytes / median plan->scalar ms_per_step (kernel-event figures: kernel_event_*)"
        roof["end_to_end_frac"] = roof["frac"]
    roof["traffic_source"] = pmc_prov
    result = {
        "metric": {"two_hop": METRIC, "triangle": TRI_METRIC, "one_hop_person": ONE_HOP_METRIC}[args.query],
        "value": count / (median_ms * 1e-3),
        "unit": "joined rows/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "int64",
        "data": (f"synthetic R-MAT s{args.scale} (Graph500 a/b/c=.57/.19/.19, edge factor {args.edge_factor}, "
                 f"seed 0x{0x5EED0000 + args.scale:X}) generated in HBM before timing"),
        "config": {
            "workload": workload_name(args),
            "scale": args.scale, "nodes": n_nodes, "rels": m, "count": count, "plan": plan,
            "id_storage": id_storage(args),
            "parallelism": "dp1",
        },
        "roofline": roof,
    }
    result["config"]["steps_mode"] = ("K single queries, each plan call -> scalar on the host between device "
                                      "syncs (SURVEY 8(d)); value = count / median")
    result["config"]["ms_per_query_median_plan_to_scalar"] = median_ms
    result["config"]["ms_per_query_mean"] = sum(times) * 1e3 / len(times)
    result["config"]["ms_per_query_min"] = min(times) * 1e3
    result["config"]["ms_per_query_max"] = max(times) * 1e3
    if pipelined_ms is not None:
        result["config"]["ms_per_step_pipelined"] = pipelined_ms
        result["config"]["joined_rows_per_s_pipelined"] = count / (pipelined_ms * 1e-3)
    result["config"]["first_query_ms"] = first_query_ms
    if "c3_handoffs" in prof:  # uint16 P3 counter hand-offs folded in by the dot kernel
        result["config"]["p3_handoffs_per_query"] = prof["c3_handoffs"]["bytes"] / prof_steps
    result["config"]["parity"] = check_fixture(args, count)
    result["config"]["lib"] = lib_digest()
    if not args.no_cpu and args.query == "two_hop":
        result["cpu_baseline"] = cpu_baseline(s, g, args.scale, args.cpu_seconds)
    if not args.no_cpu and args.query == "triangle":
        result["cpu_baseline"] = tri_cpu_baseline(s, g, args.scale, args.cpu_seconds)
    if not args.no_cpu and args.query == "one_hop_person":
        result["cpu_baseline"] = c2_cpu_baseline(g, args.scale)
        if result["cpu_baseline"]["count"] != count:
            raise SystemExit("config 2: the host count differs from the GPU count")
    print(json.dumps(result))


def run_distributed(args):
    """N ranks (torch.distributed.run), one GPU each, node-partitioned graph
    (dist.py): rank r holds the rels whose target (in-copy) and source
    (out-copy) it owns; the 2-hop count is a local partial per rank plus ONE
    int64 all-reduce over RCCL.  --layout edge: rels sharded by edge range,
    per-node histograms reduce-scattered."""
    import torch
    import torch.distributed as dist
    from capf_amd.dist import edge_range, gpu_two_hop_count, gpu_two_hop_count_sharded_async, padded_nodes
    from capf_amd.synthetic import rmat_seed, thresholds
    from capf_amd.table import GpuSession

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # RCCL prints its version banner on stdout: keep stdout for the one JSON line
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    if args.one_device:
        # rehearsal of the N-rank path on a 1-GPU box: every rank on cuda:0,
        # gloo collectives (RCCL refuses two ranks on one device)
        local = 0
        torch.cuda.set_device(0)
        dist.init_process_group("gloo")
    else:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    s = GpuSession.on_torch_stream(local)
    m = args.edge_factor << args.scale
    n_nodes = 1 << args.scale
    pipe = None  # pipelined step (node layout): enqueue into a device slot, no host read
    if args.query == "triangle":
        # config 4: the rel table replicated on every rank ("replicate the
        # rel hash set"); rank r counts its round-robin share of the oriented CSR rows
        from capf_amd.table import triangle_count_part_async
        full = s.rmat_rels(args.scale, rmat_seed(args.scale), thresholds(), 0, m)
        if not args.int64:
            full = full.compact()
        s.sync()
        partial = torch.zeros(1, dtype=torch.int64, device="cuda")

        def step():
            triangle_count_part_async(s, full, 0, n_nodes, world, rank, partial.data_ptr())
            dist.all_reduce(partial, op=dist.ReduceOp.SUM)
            return int(partial.item())
        local_rels = m
        layout = "replicated rels, oriented-CSR rows dealt round-robin over ranks; one int64 all-reduce"
        compulsory = (16.0 * m + 8.0 * n_nodes) / world
    elif args.layout == "node":
        # ingest (untimed): every rank generates the edge stream and the node range,
        # keeps its relational shards and its two count copies (dist_node_partitioned_graph)
        from capf_amd.dist_table import DistSession, GpuExchange, dist_node_partitioned_graph
        from capf_amd.graph import ElementTable, ScanGraph
        from capf_amd.planner import run
        full = s.rmat_rels(args.scale, rmat_seed(args.scale), thresholds(), 0, m)
        nodes = s.range_nodes(0, n_nodes, id_col="id")
        ds = DistSession(s, GpuExchange(s))
        g = dist_node_partitioned_graph(
            ds, ScanGraph(s, [ElementTable("node", frozenset(), nodes, {})],
                          [ElementTable("rel", frozenset(["E"]), full, {})]), compact=id_width(args))
        in_copy, out_copy = g.rel_tables[0].table.prov.info["count"].copies
        del full, nodes
        s.sync()
        q = two_hop_query()
        # the timed step: plan call → scalar through the Table SPI (planner.run on
        # DistTables; DistTable.group(∅, count(*)) dispatches the sharded count)
        step = lambda: run(g, q)[0]["count"]  # noqa: E731
        # side figure: the all-reduce of query i overlaps the kernels of query i+1
        # (RCCL stream), the copies driven directly
        pipe = lambda slot: gpu_two_hop_count_sharded_async(s, in_copy, out_copy, n_nodes, slot,  # noqa: E731
                                                            async_op=True)
        local_rels = in_copy.size + out_copy.size
        layout = (f"node-partitioned: rank holds the rels whose target (in-copy) / source (out-copy) it "
                  f"owns; the planner's 2-hop plan through DistTable; one int64 all-reduce per query")
        # rank's share of the job's compulsory bytes (src+dst int64 per rel, node ids)
        compulsory = (16.0 * m + 8.0 * n_nodes) / world
    else:
        lo, hi = edge_range(m, rank, world)
        rels = s.rmat_rels(args.scale, rmat_seed(args.scale), thresholds(), lo, hi - lo)
        if not args.int64:
            rels = rels.compact()
        npad = padded_nodes(n_nodes, world)
        hists = (torch.zeros(npad, dtype=torch.int32, device="cuda"),
                 torch.zeros(npad, dtype=torch.int32, device="cuda"))
        step = lambda: gpu_two_hop_count(s, rels, n_nodes, hists=hists)  # noqa: E731
        local_rels = hi - lo
        layout = (f"edge-range shards; per-node counts reduce-scattered over RCCL, {npad * 8} B per rank")
        compulsory = 16.0 * (hi - lo) + 8.0 * n_nodes
    count = None
    for _ in range(args.warmup):
        count = step()
    # K single queries: each starts on every rank after a barrier and ends when
    # this rank holds the all-reduced scalar; per step the slowest rank's time,
    # value from the median step (plan → scalar)
    times = []
    for _ in range(args.steps):
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        count = step()
        times.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
    dist.barrier()
    t = torch.tensor(times, dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    step_max = t.cpu().tolist()
    median_ms = statistics.median(step_max) * 1e3
    parity = check_fixture(args, count)
    pipelined_ms = None
    if pipe is not None and not args.sync_steps:
        # side figure: pipelined serving — local partial + all-reduce into slot
        # i without a host read (step i's all-reduce overlaps step i+1's
        # kernels); the K counts are checked after the closing synchronize
        slots = torch.zeros(args.steps, dtype=torch.int64, device="cuda")
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        works = [pipe(slots[i:i + 1]) for i in range(args.steps)]
        for w in works:
            w.wait()
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device="cuda")
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        pipelined_ms = float(el.item()) * 1e3 / args.steps
        got = slots.cpu().tolist()
        if any(c != count for c in got):
            raise SystemExit(f"rank {rank}: pipelined counts {got} differ from {count}")
    s.reset_profile()
    s.set_profiling(True)
    prof_steps = max(1, min(args.steps, 5))
    for _ in range(prof_steps):
        step()
    torch.cuda.synchronize()
    s.set_profiling(False)
    prof = s.profile()
    # every rank's device time per query; the JSON reports the slowest rank's
    rank_ms = sum(v["total_ms"] for k, v in prof.items() if k in PIPELINE) / prof_steps
    per_rank = torch.zeros(world, dtype=torch.float64, device="cuda")
    per_rank[rank] = rank_ms
    dist.all_reduce(per_rank, op=dist.ReduceOp.SUM)
    per_rank = per_rank.cpu().tolist()
    sys.stdout.flush()
    os.dup2(json_fd, 1)
    if rank == 0:
        ms_per_step = median_ms
        print(json.dumps({
            "metric": METRIC if args.query == "two_hop" else TRI_METRIC,
            "value": count / (median_ms * 1e-3),
            "unit": "joined rows/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "int64",
            "data": (f"synthetic R-MAT s{args.scale} (Graph500 a/b/c=.57/.19/.19, edge factor "
                     f"{args.edge_factor}), generated in HBM and partitioned before timing"),
            "config": {
                "workload": workload_name(args),
                "scale": args.scale, "nodes": n_nodes, "rels": m, "count": count,
                "rank0_rel_rows": local_rels,
                "id_storage": "int64" if args.int64 else (id_storage(args) if args.layout == "node" and args.query == "two_hop" else "FOR32"),
                "parallelism": f"dp{world} ({layout})",
                "steps_mode": ("K single queries (barrier, then local count + int64 all-reduce + "
                               "scalar on the host); per step the slowest rank, value = count / median"),
                "ms_per_query_median_plan_to_scalar": median_ms,
                "ms_per_query_max_rank_by_step": step_max,
                "ms_per_step_pipelined": pipelined_ms,
                "parity": parity,
                "device_ms_per_query_by_rank": per_rank,
                "max_rank_device_ms": max(per_rank),
                "one_device_rehearsal": bool(args.one_device),
            },
            "roofline": pipeline_roofline(prof, prof_steps, compulsory),
        }))
    dist.destroy_process_group()


def free_port():
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_ranks(args):
    """`bench.py --gpus N` started by hand (no WORLD_SIZE in the env): start N
    fresh rank processes with torch.distributed.run, one per GPU, and exit
    with the launcher's code.  This process makes no GPU call (it never
    imports the backend), so the ranks are clean children; rank 0 prints
    the JSON line on the inherited stdout."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={free_port()}",
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def fixture_count(query, scale, edge_factor):
    """The committed count for this workload (tests/golden/rmat_counts.json,
    computed by oracle/rmat.c in the dev container), or None."""
    if edge_factor != 16:
        return None
    path = os.path.join(ROOT, "tests", "golden", "rmat_counts.json")
    try:
        with open(path) as f:
            c = json.load(f)
    except OSError:
        return None
    if query == "triangle":
        return c.get("triangle", {}).get(str(scale))
    e = c.get("full", {}).get(str(scale)) or c.get("rmat", {}).get(str(scale))
    return e.get(query) if e else None


def check_fixture(args, count):
    """Parity outside the timed region: the bench's own count must be the
    fixture's (SystemExit otherwise, so no number is printed for a wrong
    answer)."""
    want = fixture_count(args.query, args.scale, args.edge_factor)
    if want is not None and count != want:
        raise SystemExit(f"count {count} != committed fixture {want} ({args.query} s{args.scale})")
    return {"fixture": want, "match": want is not None}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--scale", type=int, default=None, help="R-MAT scale (default 24; 16 for --query reach)")
    ap.add_argument("--edge-factor", type=int, default=None, help="default 16; 30 for --query reach")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--sync-steps", action="store_true",
                    help="time query-at-a-time steps only (result downloaded every step)")
    ap.add_argument("--int64", action="store_true", help="keep the id columns int64 (no FOR encoding)")
    ap.add_argument("--for32", action="store_true", help="FOR32 id columns instead of FOR24")
    ap.add_argument("--dist", action="store_true", help="distributed path even at world size 1")
    ap.add_argument("--query", choices=["two_hop", "triangle", "one_hop_person", "one_hop_rows", "var2_rows",
                                        "reach"],
                    default="two_hop",
                    help="two_hop: the headline (config 3); triangle: config 4; one_hop_person: config 2; "
                         "reach: config 5")
    ap.add_argument("--id-stride", type=int, default=1,
                    help="one_hop_rows: node ids v*stride+7 (sparse, no dense range; e.g. 1000003)")
    ap.add_argument("--one-device", action="store_true",
                    help="rehearsal: all N ranks on cuda:0 with gloo collectives (not a scaling number)")
    ap.add_argument("--layout", choices=["node", "edge"], default="node",
                    help="multi-GPU graph layout (N > 1): node-partitioned copies or edge-range shards")
    args = ap.parse_args()
    if args.scale is None:
        args.scale = 16 if args.query == "reach" else 14 if args.query == "var2_rows" else 24
    if args.edge_factor is None:
        args.edge_factor = 30 if args.query == "reach" else 16
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus and "WORLD_SIZE" in os.environ:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if args.query in ("one_hop_rows", "var2_rows"):
        run_rows_leg(args)
    elif args.query == "reach":
        run_reach_leg(args)
    elif args.gpus > 1 or world > 1 or args.dist:
        run_distributed(args)
    else:
        run_single(args)


if __name__ == "__main__":
    main()
