"""Reference-evaluated vectors for the entropy coder (tests/golden/ref_ec.npz).

    python tools/refeval/gen_ec_ref.py        (in the build container)

Runs the reference's own text through tools/refeval/rsinterp.py:

  src/ec.rs:100-600      WriterBase<WriterEncoder>: store, lr_compute, done,
                         and the Writer trait methods symbol,
                         symbol_with_update, bool, bit, literal,
                         write_golomb; native::update_cdf (:891-905)
  src/context.rs         ContextWriter::write_coeffs_lv_map (:3965-4220)
                         with write_tx_type, get_txsize_entropy_ctx,
                         txb_init_levels, get_txb_bwl, get_eob_pos_token,
                         get_nz_mag, get_nz_map_ctx_from_stats,
                         get_nz_map_ctx, get_nz_map_contexts, get_br_ctx
                         (:3419-3948), BlockContext::get_txb_ctx,
                         set_coeff_context, set_dc_sign, reset_skip_context,
                         reset_left_contexts (:1586-1868),
                         av1_get_coded_tx_size (:1949-1956), and the
                         av1_scan_orders / context statics they index.

The environment supplies: the `symbol_with_update!` macro's expansion
(`$w.symbol_with_update($s, $cdf)`, src/context.rs:1937-1947, desync_finder
off), the CDFContext fields as nested lists initialised from the default
tables exactly as CDFContext::new copies them (read from the same table text
by gen_ec_tables.py's parser), TileBlockOffset / TxSize / BlockSize /
PredictionMode values, and the `ec_window` alias (u32, src/ec.rs:20).

Vectors:
  ec_ops / ec_bytes: random operation streams (symbol_with_update on the
      default CDFs of random families, bool with random f, bit, literal,
      golomb) and the bytes `done()` returns;
  lv_*: superblock sequences in coding order (random quadtree leaves of
      64..8, skip leaves -> reset_skip_context, new superblock rows ->
      reset_left_contexts, a new tile -> a fresh BlockContext + CDFs), each
      non-skip leaf's luma / U / V transform blocks through
      write_coeffs_lv_map with random quantised coefficients, 4:2:0 and
      4:4:4; the bytes of every tile, each call's return value and stored
      context value, and the final CDFs.
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(__file__))
import gen_ec_tables as T  # noqa: E402
import gen_golden_ref as G  # noqa: E402
import rshost as H  # noqa: E402
import rsinterp as RI  # noqa: E402

REF = G.REF
ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
OUT = os.path.join(ROOT, "tests", "golden", "ref_ec.npz")

# TxSize order (src/transform/mod.rs:225-247) and BlockSize of each square
TX_NAMES = ["TX_4X4", "TX_8X8", "TX_16X16", "TX_32X32", "TX_64X64"]
BLOCK_OF_TX = [0, 3, 6, 9, 12]  # BLOCK_4X4, 8X8, 16X16, 32X32, 64X64 (src/partition.rs:116-140)
NEARESTMV = 14  # PredictionMode (src/predict.rs:135-165)


def u16(v):
    return RI.TInt(int(v), "u16")


class TxSq(int):
    """A square TxSize value (src/transform/mod.rs:162-360)."""

    def __new__(cls, idx):
        return int.__new__(cls, idx)

    def width(self):
        return RI.TInt(4 << int(self), "usize")

    height = width

    def width_mi(self):
        return RI.TInt(1 << int(self), "usize")

    height_mi = width_mi

    def width_log2(self):
        return RI.TInt(int(self) + 2, "usize")

    height_log2 = width_log2

    def area_log2(self):
        return RI.TInt(2 * (int(self) + 2), "usize")

    def area(self):
        return RI.TInt(1 << (2 * (int(self) + 2)), "usize")

    def sqr(self):
        return self

    def sqr_up(self):
        return self

    def block_size(self):
        return H.BlockSizeV(BLOCK_OF_TX[int(self)])


def tile_bo(x, y):
    bo = RI.Struct("BlockOffset", {"x": RI.TInt(x, "usize"), "y": RI.TInt(y, "usize")})
    return RI.Struct("TileBlockOffset", {"0": bo, "y_in_sb": lambda: RI.TInt(y & 15, "usize")})


def make():
    I = G.make_interp()
    for extra in ("ec.rs", "context.rs", "partition.rs"):
        s = RI.Source(REF + extra)
        if extra == "ec.rs":  # `type ec_window = u32;` (src/ec.rs:20)
            s.src = s.src.replace("ec_window", "u32")
        I.sources.append(s)
    ec = G.src_of(I, "ec.rs")
    for after in ("impl StorageBackend for WriterBase<WriterEncoder>", "impl<S> WriterBase<S>",
                  "impl WriterBase<WriterEncoder>", "impl<S> Writer for WriterBase<S>"):
        I.define_impl("WriterBase", ec.impl("WriterBase", after))
    ctx = G.src_of(I, "context.rs")
    I.define_impl("BlockContext", [ctx.fn(n, "impl<'a> BlockContext<'a>") for n in (
        "set_dc_sign", "set_coeff_context", "reset_left_coeff_context", "reset_skip_context",
        "reset_left_contexts", "get_txb_ctx", "reset_left_partition_context",
        "reset_left_tx_context")])
    I.define_impl("ContextWriter", [ctx.fn(n, "impl<'a> ContextWriter<'a>") for n in (
        "write_coeffs_lv_map", "write_tx_type", "get_txsize_entropy_ctx", "txb_init_levels",
        "get_txb_bwl", "get_eob_pos_token", "get_nz_mag", "get_nz_map_ctx_from_stats",
        "get_nz_map_ctx", "get_nz_map_contexts", "get_br_ctx")])
    env = I.globals.vars
    for i, n in enumerate(TX_NAMES):
        env[n] = TxSq(i)
    for i, n in enumerate(["4X8", "8X4", "8X16", "16X8", "16X32", "32X16", "32X64", "64X32",
                           "4X16", "16X4", "8X32", "32X8", "16X64", "64X16"]):
        env["TX_" + n] = 5 + i  # rectangular sizes: only compared against (never coded here)
    env["TxSize"] = type("TxSizeNS", (), {n: TxSq(i) for i, n in enumerate(TX_NAMES)})
    env["TxSet"] = type("TxSetNS", (), {"TX_SET_DCTONLY": 0, "TX_SET_DCT_IDTX": 1,
                                        "TX_SET_DTT4_IDTX": 2,
                                        "TX_SET_DTT4_IDTX_1DDCT_16X16": 3,
                                        "TX_SET_DTT4_IDTX_1DDCT": 4, "TX_SET_DTT9_IDTX": 5,
                                        "TX_SET_DTT9_IDTX_1DDCT": 6, "TX_SET_ALL16_16X16": 7,
                                        "TX_SET_ALL16": 8})
    for i, n in enumerate(("TX_CLASS_2D", "TX_CLASS_HORIZ", "TX_CLASS_VERT")):
        env[n] = i
    env["PredictionMode"] = type("PM", (), {"NEARESTMV": NEARESTMV})
    for i, n in enumerate(H.BLOCK_NAMES):
        env["BLOCK_" + n] = H.BlockSizeV(i)

    def subsampled_size(b, xdec, ydec):  # src/partition.rs subsampled_size (square blocks)
        return H.BlockSizeV(H.BLOCK_NAMES.index("%dX%d" % (max(4, b.w >> int(xdec)),
                                                           max(4, b.h >> int(ydec)))))
    H.BlockSizeV.subsampled_size = subsampled_size
    env["TXB_CTX"] = RI.StructType("TXB_CTX", {"txb_skip_ctx": "usize", "dc_sign_ctx": "usize"})
    env["AlignedArray"] = G.AlignedArray
    env["WriterEncoder"] = RI.StructType("WriterEncoder")
    env["WriterBase"] = RI.StructType("WriterBase")
    env["BlockContext"] = RI.StructType("BlockContext")
    env["ContextWriter"] = RI.StructType("ContextWriter")

    def m_swu(interp, args, e):  # symbol_with_update!($self, $w, $s, $cdf)
        return interp.ev(("mcall", args[1], "symbol_with_update", [args[2], args[3]], None), e)
    I.macros = {"symbol_with_update": m_swu}
    I.release = True
    return I


def cdf_fields(qctx):
    """CDFContext's coefficient fields as CDFContext::new builds them
    (src/context.rs:793-850), from the default tables' text."""
    tok = T.strip_comments(open(os.path.join(REF, "token_cdfs.rs")).read())
    em = T.strip_comments(open(os.path.join(REF, "entropymode.rs")).read())

    def typed(v):
        return [typed(x) for x in v] if isinstance(v, list) else u16(v)
    f = {}
    for field, st in (("txb_skip_cdf", "av1_default_txb_skip_cdfs"),
                      ("dc_sign_cdf", "av1_default_dc_sign_cdfs"),
                      ("eob_extra_cdf", "av1_default_eob_extra_cdfs"),
                      ("eob_flag_cdf16", "av1_default_eob_multi16_cdfs"),
                      ("eob_flag_cdf32", "av1_default_eob_multi32_cdfs"),
                      ("eob_flag_cdf64", "av1_default_eob_multi64_cdfs"),
                      ("eob_flag_cdf128", "av1_default_eob_multi128_cdfs"),
                      ("eob_flag_cdf256", "av1_default_eob_multi256_cdfs"),
                      ("eob_flag_cdf512", "av1_default_eob_multi512_cdfs"),
                      ("eob_flag_cdf1024", "av1_default_eob_multi1024_cdfs"),
                      ("coeff_base_eob_cdf", "av1_default_coeff_base_eob_multi_cdfs"),
                      ("coeff_base_cdf", "av1_default_coeff_base_multi_cdfs"),
                      ("coeff_br_cdf", "av1_default_coeff_lps_multi_cdfs")):
        f[field] = typed(T.parse_static(tok, st)[qctx])
    f["inter_tx_cdf"] = typed(T.parse_static(em, "default_inter_ext_tx_cdf"))
    return f


FLAT_ORDER = ["txb_skip_cdf", "eob_flag_cdf16", "eob_flag_cdf32", "eob_flag_cdf64",
              "eob_flag_cdf128", "eob_flag_cdf256", "eob_flag_cdf512", "eob_flag_cdf1024",
              "eob_extra_cdf", "coeff_base_eob_cdf", "coeff_base_cdf", "coeff_br_cdf",
              "dc_sign_cdf", "inter_tx_cdf"]


def flatten_cdfs(fc):
    return [int(v) for n in FLAT_ORDER for v in T.flat(fc[n])]


def new_writer():
    return RI.Struct("WriterBase", {"rng": RI.TInt(0x8000, "u16"), "cnt": RI.TInt(-9, "i16"),
                                    "fake_bits_frac": RI.TInt(0, "u32"),
                                    "s": RI.Struct("WriterEncoder", {"precarry": [],
                                                                     "low": RI.TInt(0, "u32")})})


def call(I, obj, name, *args):
    return I.make_method(obj._name, name, obj, I.globals)(*args)


# ------------------------------------------------------------- range coder
def gen_writer(I, rng, out, nstreams=24):
    fams = [(n, e) for n, _, shape, e in T.FAMILIES]
    ops_all, bytes_all, idx = [], [], []
    for si in range(nstreams):
        q = int(rng.integers(0, 4))
        if q not in G_TABLE_CACHE:
            G_TABLE_CACHE[q] = flatten_cdfs(cdf_fields(q))
        flat_tab = G_TABLE_CACHE[q]
        state = list(flat_tab)
        w = new_writer()
        ops = []
        n = int(rng.integers(20, 400))
        offs = {nm: o for nm, o in zip([f[0] for f in T.FAMILIES], _fam_offsets())}
        for _ in range(n):
            k = int(rng.integers(0, 10))
            if k < 5:  # symbol_with_update on one CDF of a family
                nm, e = fams[int(rng.integers(0, len(fams)))]
                cnt = _fam_count(nm)
                ci = int(rng.integers(0, cnt))
                o = offs[nm] + ci * e
                s = int(rng.integers(0, e - 1))
                cdf = [RI.TInt(v, "u16") for v in state[o:o + e]]
                call(I, w, "symbol_with_update", RI.TInt(s, "u32"), cdf)
                state[o:o + e] = [int(v) for v in cdf]
                ops.append((0, q, o, e, s))
            elif k < 7:
                f = int(rng.integers(1, 32768))
                b = int(rng.integers(0, 2))
                call(I, w, "bool", bool(b), RI.TInt(f, "u16"))
                ops.append((1, f, b, 0, 0))
            elif k < 8:
                b = int(rng.integers(0, 2))
                call(I, w, "bit", RI.TInt(b, "u16"))
                ops.append((2, b, 0, 0, 0))
            elif k < 9:
                nb = int(rng.integers(1, 17))
                v = int(rng.integers(0, 1 << nb))
                call(I, w, "literal", RI.TInt(nb, "u8"), RI.TInt(v, "u32"))
                ops.append((3, nb, v, 0, 0))
            else:
                v = int(rng.integers(0, 3000)) if rng.integers(0, 4) else int(rng.integers(0, 65534))
                call(I, w, "write_golomb", RI.TInt(v, "u16"))
                ops.append((4, v, 0, 0, 0))
        b = call(I, w, "done")
        idx.append((len(ops_all), len(ops), len(bytes_all), len(b)))
        ops_all += ops
        bytes_all += [int(x) for x in b]
    out["ec_ops"] = np.array(ops_all, np.int32)
    out["ec_bytes"] = np.array(bytes_all, np.uint8)
    out["ec_index"] = np.array(idx, np.int64)
    print("ec: %d streams, %d ops, %d bytes" % (nstreams, len(ops_all), len(bytes_all)))


G_TABLE_CACHE = {}


def _fam_offsets():
    o, out = 0, []
    for n, _, shape, e in T.FAMILIES:
        out.append(o)
        c = e
        for d in shape:
            c *= d
        o += c
    return out


def _fam_count(name):
    for n, _, shape, e in T.FAMILIES:
        if n == name:
            c = 1
            for d in shape:
                c *= d
            return c
    raise KeyError(name)


# ------------------------------------------------------- coefficient coding
def rand_coeffs(rng, cw, scale):
    """Quantised coefficients of a coded cw x cw transform: a decaying
    Laplacian in raster order, mostly small, some large (golomb range),
    some blocks all zero."""
    if rng.random() < 0.15:
        return np.zeros(cw * cw, np.int64)
    r = np.arange(cw)
    decay = np.exp(-(r[:, None] + r[None, :]) / (cw * rng.uniform(0.05, 0.6)))
    c = np.round(rng.laplace(0, scale, (cw, cw)) * decay).astype(np.int64)
    if rng.random() < 0.3:  # a few big ones
        k = int(rng.integers(1, 4))
        for _ in range(k):
            c[int(rng.integers(0, min(cw, 6))), int(rng.integers(0, min(cw, 6)))] = int(
                rng.integers(-3000, 3000))
    if rng.random() < 0.2:  # a sparse block
        c[np.abs(c) < 3] = 0
    return c.reshape(-1)


def leaves(rng, x4, y4, lg, minlg, vis_w4, vis_h4, out):
    """Quadtree leaves in z-order (luma 4x4 units; lg = log2 size px)."""
    if x4 >= vis_w4 or y4 >= vis_h4:
        return
    n4 = 1 << (lg - 2)
    must = x4 + n4 > vis_w4 or y4 + n4 > vis_h4
    if lg > minlg and (must or rng.random() < 0.45):
        h = n4 // 2
        for dy in (0, h):
            for dx in (0, h):
                leaves(rng, x4 + dx, y4 + dy, lg - 1, minlg, vis_w4, vis_h4, out)
    else:
        out.append((x4, y4, lg))


def gen_lv(I, rng, out):
    jobs, coeffs, rets, tile_bytes, cases, finals = [], [], [], [], [], []
    nc = 0
    case_id = 0
    for xdec, ydec in ((1, 1), (0, 0)):
        for trial in range(3 if xdec else 2):
            q = int(rng.integers(0, 4))
            sbw, sbh = (2, 2) if trial < 2 else (3, 1)
            vis_w4 = sbw * 16 - (int(rng.integers(0, 3)) * 2 if trial == 1 else 0)
            vis_h4 = sbh * 16 - (int(rng.integers(1, 4)) * 2 if trial == 1 else 0)
            ntiles = 2 if trial == 0 else 1
            j0 = len(jobs)
            fc0 = None
            for tile in range(ntiles):
                jobs.append((3, 0, 0, 0, 0, 0, 0, 0, 0, 0))
                fc = cdf_fields(q)
                if fc0 is None:
                    fc0 = flatten_cdfs(fc)
                bc = RI.Struct("BlockContext", {
                    "above_coeff_context": [[RI.TInt(0, "u8")] * 1024 for _ in range(3)],
                    "left_coeff_context": [[RI.TInt(0, "u8")] * 16 for _ in range(3)],
                    "left_partition_context": [RI.TInt(0, "u8")] * 8,
                    "left_tx_context": [RI.TInt(0, "u8")] * 16})
                cw_obj = RI.Struct("ContextWriter", {"bc": bc, "fc": RI.Struct("CDFContext", fc)})
                w = new_writer()
                rets.append(0)
                for sby in range(sbh):
                    jobs.append((2, 0, 0, 0, 0, 0, 0, 0, 0, 0))
                    call(I, bc, "reset_left_contexts")
                    rets.append(0)
                    for sbx in range(sbw):
                        lv = []
                        leaves(rng, sbx * 16, sby * 16, 6, 3, vis_w4, vis_h4, lv)
                        for (x4, y4, lg) in lv:
                            bo = tile_bo(x4, y4)
                            if rng.random() < 0.3:  # a skip leaf
                                call(I, bc, "reset_skip_context", bo, H.BlockSizeV(BLOCK_OF_TX[lg - 2]),
                                     RI.TInt(xdec, "usize"), RI.TInt(ydec, "usize"))
                                jobs.append((1, 0, x4, y4, 0, 0, 0, lg, lg, 0))
                                rets.append(0)
                                continue
                            intra = lg == 6 and rng.random() < 0.25
                            mode = RI.TInt(0 if intra else NEARESTMV, "usize")
                            for p in range(3):
                                xd, yd = (xdec, ydec) if p else (0, 0)
                                plg = lg - xd  # square blocks: w and h decimate alike here
                                tx = min(plg - 2, 4)
                                if p and xdec == 0 and lg == 6:
                                    tx = 3  # 4:4:4 64x64 chroma: four 32x32 (largest_chroma_tx_size)
                                cwid = min(4 << tx, 32)
                                n_tx = 4 if (p and xdec == 0 and lg == 6) else 1
                                for t in range(n_tx):
                                    tx4x = x4 + (t % 2) * 8 if n_tx == 4 else x4
                                    tx4y = y4 + (t // 2) * 8 if n_tx == 4 else y4
                                    c = rand_coeffs(rng, cwid, 6.0 if p == 0 else 3.0)
                                    cin = [RI.TInt(int(v), "i32") for v in c]
                                    # chroma: write_tx_tree passes uv_tx_type = DCT_DCT, bsize
                                    # subsampled; tx_bo per chroma tx block (src/encoder.rs:1997-2003)
                                    has = call(I, cw_obj, "write_coeffs_lv_map", w, RI.TInt(p, "usize"),
                                               tile_bo(tx4x, tx4y), RI.Slice(cin), mode, TxSq(tx),
                                               RI.TInt(0, "usize"), H.BlockSizeV(BLOCK_OF_TX[plg - 2]),
                                               RI.TInt(xd, "usize"), RI.TInt(yd, "usize"), True)
                                    cul = int(bc.above_coeff_context[p][(tx4x >> xd)])
                                    jobs.append((0, p, tx4x, tx4y, tx, 0, 0 if intra else 1, plg, plg, nc))
                                    coeffs += [int(v) for v in c]
                                    nc += len(c)
                                    rets.append(int(bool(has)) | cul << 1)
                b = call(I, w, "done")
                tile_bytes.append(len(b))
                out.setdefault("_bytes", []).extend(int(x) for x in b)
                finals.append(flatten_cdfs(fc))
            cases.append((case_id, j0, len(jobs) - j0, xdec, ydec, q, ntiles))
            case_id += 1
            out.setdefault("_init", []).append(fc0)
    out["lv_jobs"] = np.array(jobs, np.int32)
    out["lv_coeffs"] = np.array(coeffs, np.int32)
    out["lv_ret"] = np.array(rets, np.int32)
    out["lv_tile_bytes"] = np.array(tile_bytes, np.int32)
    out["lv_bytes"] = np.array(out.pop("_bytes"), np.uint8)
    out["lv_cases"] = np.array(cases, np.int32)
    out["lv_final_cdf"] = np.array(finals, np.uint16)
    out["lv_init_cdf"] = np.array(out.pop("_init"), np.uint16)
    print("lv: %d cases, %d jobs, %d coefficient blocks, %d bytes" % (
        len(cases), len(jobs), sum(1 for j in jobs if j[0] == 0), len(out["lv_bytes"])))


def main():
    t0 = time.time()
    rng = np.random.default_rng(0xEC)
    out = {}
    gen_writer(make(), rng, out)
    gen_lv(make(), rng, out)  # a fresh evaluator
    np.savez_compressed(OUT, **out)
    print("wrote %s in %.0f s" % (OUT, time.time() - t0))


if __name__ == "__main__":
    main()
