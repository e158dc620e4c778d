"""Builds tests/golden/okapi_api.json from the reference's Scala sources: for
every okapi name the JVM drop-in (integration/scala) imports or matches on,
its definitions (kind, case-class arity); for every okapi trait / class the
drop-in extends, its declared members and parents (transitively).  Names and
arities only — no source text is kept.

    python tests/golden/make_okapi_api.py [/root/reference]
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import okapi_scala_scan as sc  # noqa: E402

OUT = os.path.join(HERE, "okapi_api.json")


def build(ref_root):
    idx = sc.index_reference(ref_root)
    srcs = sc.integration_sources()
    names, wild = {}, {}
    for text in srcs.values():
        for prefix, name in sc.imports(text):
            if name == "_":
                wild[prefix] = sorted(sc.package_names(idx, prefix))
            else:
                names[f"{prefix}.{name}"] = sc.resolve(idx, prefix, name)
    # extractor names of wildcard-imported packages
    for text in srcs.values():
        calls, bare = sc.patterns(text)
        for n in [c for c, _ in calls] + bare:
            for prefix, defined in wild.items():
                if n in defined:
                    names[f"{prefix}.{n}"] = sc.resolve(idx, prefix, n)
    # members of the okapi parents, transitively (each parent looked up where
    # its child imports it from, then next to its child)
    where = {q.rsplit(".", 1)[1]: q.rsplit(".", 1)[0] for q in names}
    todo = []
    for text in srcs.values():
        for cls, (parents, _) in sc.classes(text).items():
            todo += [(p, where[p], None) for p in parents if p in where]
    members, seen = {}, set()
    while todo:
        p, prefix, near = todo.pop()
        if p in seen:
            continue
        seen.add(p)
        info = sc.members_of(idx, p, prefix, near)
        if info is None:
            continue
        members[p] = {"members": info[0], "parents": info[1]}
        todo += [(q, None, info[2]) for q in info[1]]
    return {"reference": "soerenreichardt/cypher-for-apache-flink (okapi main sources)",
            "names": {k: [list(d) for d in v] for k, v in sorted(names.items())},
            "wildcard_packages": {k: v for k, v in sorted(wild.items())},
            "members": dict(sorted(members.items()))}


if __name__ == "__main__":
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    data = build(ref)
    with open(OUT, "w") as f:
        json.dump(data, f, indent=1, sort_keys=True)
    print(f"{OUT}: {len(data['names'])} names, {len(data['members'])} parent types")
