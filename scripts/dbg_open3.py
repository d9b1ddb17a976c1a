"""Debug helper: repeat the parity test's seal/open batches in one process and
report every mismatching record (index, length, status)."""
import os, sys, random
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import pyoracle as po
import talos_amd as ta
from talos_amd.batch import RecordBatch
import test_gpu_parity as T

ta.load_library()
oracle = po.Oracle()
eng = ta.Engine(0)
prev = None
keep = []
if os.environ.get("IMPL"): ta.set_gcm_impl(os.environ["IMPL"])
for it in range(int(os.environ.get("ITERS", "12"))):
    kind = [po.AES_128_GCM, po.AES_256_GCM][it % 2]
    rnd = random.Random(21 + it)
    kinds = [kind] * 2
    params = T._mk_sessions(ta, rnd, kinds)
    table = ta.SessionTable(eng, len(params)); table.install(0, params)
    osess = T._oracle_sessions(oracle, params)
    recs = T._records(rnd, len(params), T.LENGTHS, kinds, True)
    sb = RecordBatch(eng, recs, "seal"); sb.run(table)
    bodies, bad = [], []
    for i, ((st, body), (sid, seq, rt, pt, k)) in enumerate(zip(sb.results(), recs)):
        exp = oracle.tls_seal(osess[sid], seq, rt, pt)
        bodies.append(exp)
        if body != exp:
            d = [j for j in range(min(len(body), len(exp))) if body[j] != exp[j]]
            why = "?"
            if prev is not None:
                posess, precs = prev
                if oracle.tls_seal(posess[sid], seq, rt, pt) == body:
                    why = "prev-session-keys"
                elif i < len(precs) and oracle.tls_seal(osess[sid], precs[i][1], rt, pt)[8:] == body[8:]:
                    why = "prev-seq"
            if len(pt) >= 256 and os.environ.get("KSDIAG"):
                kt = bytes(a ^ b for a, b in zip(exp[8:8 + len(pt)], pt))
                kg = bytes(a ^ b for a, b in zip(body[8:8 + len(pt)], pt))
                blocks = {kt[16 * q:16 * q + 16]: q for q in range(len(pt) // 16)}
                m = [(q, blocks.get(kg[16 * q:16 * q + 16])) for q in range(len(pt) // 16)]
                okb = sum(1 for q, v in m if v == q)
                print("  ksdiag rec", i, "len", len(pt), "blocks ok", okb, "of", len(m),
                      "first bad", [(q, v) for q, v in m if v != q][:6], flush=True)
            bad.append(("seal", i, len(pt), st, d[:1], len(d), why))
    orecs = [(sid, seq, rt, b, k) for (sid, seq, rt, pt, k), b in zip(recs, bodies)]
    ob = RecordBatch(eng, orecs, "open"); ob.run(table)
    for i, ((st, got), (sid, seq, rt, pt, k)) in enumerate(zip(ob.results(), recs)):
        if st != len(pt) or got != pt:
            bad.append(("open", i, len(pt), st))
    dd = os.environ.get("TLSGPU_DBG_DUMP_PRE")
    if dd and bad:
        import glob
        fs = sorted(glob.glob(dd + "/pre_1_*.bin"), key=lambda f: os.path.getmtime(f))
        raw = open(fs[-1], "rb").read()
        nbad = 0
        for i, (sid, seq, rt, pt, k) in enumerate(recs):
            p = params[sid]
            j0 = bytes(p.fixed_iv) + seq.to_bytes(8, "big") + (1).to_bytes(4, "big")
            ek0 = oracle.aes_encrypt(bytes(p.key), j0)
            got = raw[48 * i:48 * i + 16]
            if got != ek0:
                nbad += 1
                if nbad <= 3:
                    alt = [q for q in range(len(recs)) if raw[48 * q:48 * q + 16] == got]
                    print("  pre ek0 mismatch rec", i, "sid", sid, got.hex(), ek0.hex(), "same as recs", alt, flush=True)
        print("  pre file", fs[-1], "ek0 mismatches", nbad, flush=True)
    print("iter", it, "kind", kind, "records", len(recs), "bad", bad[:8], len(bad), flush=True)
    if not os.environ.get("NOFREE"):
        table.close(); sb.free(); ob.free()
    else:
        keep.append((table, sb, ob))
    prev = (osess, recs)
