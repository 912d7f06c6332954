"""Generate tests/golden/reassemble.json from the REFERENCE's own rx stack (dev container only).

    make -C oracle ref && python tests/golden/make_reasm_golden.py

For every stream of tests/reasm_cases.py, the reference's reactor + stream hook
(oracle/reactor_harness.c driving NetReactor_handle -> on_read_stream -> fragment cache ->
on_recv, compiled from /root/reference by oracle/Makefile `ref`, websocket glue around the
reference's websocketframeDecode) delivers the stream fed through a socketpair; the delivered
messages are recorded as data: their lengths and a SHA-256 of their bodies back to back, the
bytes and frames the reactor loop consumed, the detach error and the fragment-cache state at
the end. The deliveries must not depend on how the stream is split into reads: every case
runs at several write sizes and all must agree.

Only data is committed (stream hashes, lengths, digests); no reference source.
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import reasm_cases as R  # noqa: E402
import ref_reactor as X  # noqa: E402


def main():
    assert X.available(), "build the reference first: make -C oracle ref"
    out = {"generator": "tests/golden/make_reasm_golden.py (reference rx stack: oracle/reactor_harness.c)",
           "glue": "on_decode = websocketframeDecode; err if ret<0, incomplete if 0, else decodelen=ret, "
                   "bodyptr=data, bodylen=(unsigned)datalen, fragment_eof=is_fin, pktype=NETPACKET_FRAGMENT",
           "cases": []}
    for name in R.CASES:
        wire, limit = R.build(name)
        runs = []
        for chunk in (7, 1500, 65536, len(wire) + 1):
            if chunk == 7 and len(wire) > 200000:
                continue
            r = X.reactor_deliver(wire, chunk, limit)
            runs.append((chunk, r))
        r0 = runs[0][1]
        for chunk, r in runs[1:]:
            assert r["lens"] == r0["lens"] and (r["bodies"] == r0["bodies"]).all(), (name, chunk)
            for k in ("consumed", "frames", "detach_error", "pending", "cached"):
                assert r[k] == r0[k], (name, chunk, k)
        out["cases"].append({
            "name": name, "wire_len": len(wire), "wire_sha256": R.sha256(wire), "readcache_max": limit,
            "write_sizes": [c for c, _ in runs],
            "msg_lens": r0["lens"], "bodies_sha256": R.sha256(r0["bodies"]),
            "consumed": r0["consumed"], "frames": r0["frames"], "detach_error": r0["detach_error"],
            "pending": r0["pending"], "cached": r0["cached"]})
        print(name, len(r0["lens"]), "messages, consumed", r0["consumed"], "of", len(wire), "detach",
              r0["detach_error"], "pending", r0["pending"], r0["cached"])
    with open(os.path.join(HERE, "reassemble.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
