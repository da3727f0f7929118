// CauseWeave.java -- the JVM side of the drop-in boundary (include/causeweave.h).
//
// Panama FFM (JDK 22+) downcalls into libcauseweave.so, plus the marshalling the
// C ABI asks of its host: site-ids interned per document in String.compareTo
// order (the order clojure.core/compare gives ids, util.cljc:4-10), ids packed
// as K64 keys when they fit 63 bits and as K128 (hi = ts, lo = site << 32 | tx)
// otherwise, the root [[0 "0" 0] nil nil] flagged, the special values
// (shared.cljc:21) as kinds.  causal/collections/list_gpu.cljc turns the results
// back into the reference's ct maps.
//
// Not compiled or run in this repository's image (no JDK); the Python twin of
// every call here is cause_amd/abi.py + cause_amd/pack.py, which the tests run.
package causal.gpu;

import java.lang.foreign.Arena;
import java.lang.foreign.FunctionDescriptor;
import java.lang.foreign.Linker;
import java.lang.foreign.MemoryLayout;
import java.lang.foreign.MemorySegment;
import java.lang.foreign.StructLayout;
import java.lang.foreign.SymbolLookup;
import java.lang.invoke.MethodHandle;
import java.util.ArrayList;
import java.util.Arrays;
import java.util.List;
import java.util.TreeSet;

import static java.lang.foreign.ValueLayout.ADDRESS;
import static java.lang.foreign.ValueLayout.JAVA_BYTE;
import static java.lang.foreign.ValueLayout.JAVA_INT;
import static java.lang.foreign.ValueLayout.JAVA_LONG;

public final class CauseWeave implements AutoCloseable {
  // ---- constants of include/causeweave.h ----
  public static final long CW_NIL = -1L;            // UINT64_MAX
  public static final long NON_ID_CAUSE = -2L;      // a list cause that is not an id
  public static final int KIND_NORMAL = 0, KIND_HIDE = 1, KIND_HHIDE = 2, KIND_HSHOW = 3,
      KIND_ROOT = 4;
  public static final int STATUS_ROOT = 1, STATUS_DUP = 2, STATUS_ORPHAN = 4,
      STATUS_NON_LAMPORT = 8, STATUS_MAP_KEY = 16, STATUS_INTERNAL = 32, STATUS_WEFT = 64,
      STATUS_KEY_RANGE = 128;
  static final int CW_MEM_HOST = 0;

  // ---- struct layouts (x86-64, natural alignment) ----
  static final StructLayout LIST_BATCH = MemoryLayout.structLayout(
      JAVA_LONG.withName("n_docs"), ADDRESS.withName("doc_offsets"), ADDRESS.withName("id_key"),
      ADDRESS.withName("cause_key"), ADDRESS.withName("kind"), JAVA_INT.withName("key_bits"),
      JAVA_INT.withName("ts_shift"), JAVA_INT.withName("site_shift"), JAVA_INT.withName("site_bits"));
  static final StructLayout LIST_BATCH_K128 = MemoryLayout.structLayout(
      JAVA_LONG.withName("n_docs"), ADDRESS.withName("doc_offsets"), ADDRESS.withName("id_key"),
      ADDRESS.withName("cause_key"), ADDRESS.withName("kind"));
  static final StructLayout LIST_RESULT = MemoryLayout.structLayout(
      ADDRESS.withName("weave_perm"), ADDRESS.withName("visible_bits"),
      ADDRESS.withName("visible_count"), ADDRESS.withName("max_ts"), ADDRESS.withName("status"),
      ADDRESS.withName("yarn_perm"));
  static final StructLayout MAP_BATCH = MemoryLayout.structLayout(
      JAVA_LONG.withName("n_colls"), ADDRESS.withName("coll_offsets"), ADDRESS.withName("id_key"),
      ADDRESS.withName("cause"), ADDRESS.withName("cause_is_id"), ADDRESS.withName("kind"),
      JAVA_INT.withName("key_bits"), JAVA_INT.withName("token_bits"));
  static final StructLayout MAP_RESULT = MemoryLayout.structLayout(
      JAVA_LONG.withName("cap_segs"), JAVA_LONG.withName("n_segs"), ADDRESS.withName("seg_offsets"),
      ADDRESS.withName("seg_coll"), ADDRESS.withName("seg_key"), ADDRESS.withName("seg_active"),
      ADDRESS.withName("seg_perm"), ADDRESS.withName("status"));

  // ---- downcalls ----
  static final Linker LINKER = Linker.nativeLinker();
  static final SymbolLookup LIB =
      SymbolLookup.libraryLookup(System.getProperty("causeweave.lib", "libcauseweave.so"),
                                 Arena.global());

  static MethodHandle h(String name, FunctionDescriptor d) {
    return LINKER.downcallHandle(LIB.find(name).orElseThrow(), d);
  }

  static final MethodHandle CTX_CREATE =
      h("cw_ctx_create", FunctionDescriptor.of(JAVA_INT, JAVA_INT, ADDRESS));
  static final MethodHandle CTX_DESTROY = h("cw_ctx_destroy", FunctionDescriptor.ofVoid(ADDRESS));
  static final MethodHandle LAST_ERROR =
      h("cw_last_error", FunctionDescriptor.of(ADDRESS, ADDRESS));
  static final MethodHandle WEAVE_LISTS =
      h("cw_weave_lists", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, ADDRESS, JAVA_INT));
  static final MethodHandle WEAVE_LISTS_K128 =
      h("cw_weave_lists_k128", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, ADDRESS, JAVA_INT));
  static final MethodHandle WEAVE_MAPS =
      h("cw_weave_maps", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, ADDRESS, JAVA_INT));

  private final MemorySegment ctx;

  /** cw_ctx_create on HIP device `device`.  A context is used by one thread at a time
   *  (the Clojure side keeps one per thread, list_gpu.cljc). */
  public CauseWeave(int device) throws Throwable {
    try (Arena a = Arena.ofConfined()) {
      MemorySegment out = a.allocate(ADDRESS);
      if ((int) CTX_CREATE.invokeExact(device, out) != 0)
        throw new IllegalStateException("cw_ctx_create: no usable HIP device " + device);
      ctx = out.get(ADDRESS, 0);
    }
  }

  @Override
  public void close() throws Throwable {
    CTX_DESTROY.invokeExact(ctx);
  }

  private void check(int rc, String what) throws Throwable {
    if (rc != 0) {
      MemorySegment msg = (MemorySegment) LAST_ERROR.invokeExact(ctx);
      throw new IllegalStateException(what + ": " + msg.reinterpret(4096).getString(0));
    }
  }

  // =========================================================== marshalling ====
  /** One node: id = (ts, site, tx); cause = an id (causeKind 0), nil (1) or a
   *  value that is not an id, e.g. a map key (2); kind = KIND_*. */
  public static final class Node {
    public final long ts, tx, cts, ctx;
    public final String site, csite;
    public final int causeKind, kind;

    public Node(long ts, String site, long tx, int causeKind, long cts, String csite, long ctx,
                int kind) {
      this.ts = ts; this.site = site; this.tx = tx; this.causeKind = causeKind;
      this.cts = cts; this.csite = csite; this.ctx = ctx; this.kind = kind;
    }
  }

  /** Results of one document, indices into the document's node list. */
  public static final class ListResult {
    public int[] weavePerm;     // weave order
    public boolean[] rendered;  // per weave position: not hide? (list.cljc:48-55)
    public int visibleCount;    // (count list), list.cljc:77
    public long maxTs;          // ::lamport-ts after refresh-ts (shared.cljc:243-249)
    public int status;          // STATUS_*
    public int[] yarnPerm;      // ::yarns: by site (String.compareTo), id-ascending
  }

  /** Site ranks of one document in String.compareTo order (UTF-16 code units),
   *  over every site in an id or an id-cause. */
  static String[] internSites(List<Node> doc) {
    TreeSet<String> s = new TreeSet<>();  // natural order of String = compareTo
    for (Node n : doc) {
      s.add(n.site);
      if (n.causeKind == 0) s.add(n.csite);
    }
    return s.toArray(new String[0]);
  }

  static int bits(long v) { return v == 0 ? 0 : 64 - Long.numberOfLeadingZeros(v); }

  /** Full reweave of a batch of list documents (c.list/weave 1-arity,
   *  list.cljc:26-28, plus spin / refresh-ts / hide?).  K64 when every id
   *  fits 63 bits, K128 otherwise. */
  public ListResult[] weaveLists(List<List<Node>> docs) throws Throwable {
    int D = docs.size();
    long N = 0, mts = 0, mtx = 0;
    int msite = 0;
    List<String[]> ranks = new ArrayList<>(D);
    for (List<Node> d : docs) {
      String[] r = internSites(d);
      ranks.add(r);
      msite = Math.max(msite, r.length - 1);
      for (Node n : d) {
        if (n.ts < 0 || n.tx < 0) throw new IllegalArgumentException("negative ts / tx-index");
        mts = Math.max(mts, n.ts);
        mtx = Math.max(mtx, n.tx);
        if (n.causeKind == 0) {
          mts = Math.max(mts, n.cts);
          mtx = Math.max(mtx, n.ctx);
        }
      }
      N += d.size();
    }
    // at least one site bit: the ids are packed with the same width the yarn
    // partition (site_bits) reads, also when every node is on site "0"
    int tsBits = bits(mts), siteBits = Math.max(bits(msite), 1), txBits = bits(mtx);
    boolean k128 = tsBits + siteBits + txBits > 63;
    if (k128 && (siteBits > 32 || txBits > 32))
      throw new IllegalArgumentException("ids do not fit K128 (site ranks and tx < 2^32)");
    int w = k128 ? 2 : 1;
    try (Arena a = Arena.ofConfined()) {
      MemorySegment off = a.allocate(JAVA_LONG, D + 1);
      MemorySegment id = a.allocate(JAVA_LONG, Math.max(1, N * w));
      MemorySegment cause = a.allocate(JAVA_LONG, Math.max(1, N * w));
      MemorySegment kind = a.allocate(JAVA_BYTE, Math.max(1, N));
      long j = 0;
      for (int d = 0; d < D; d++) {
        off.setAtIndex(JAVA_LONG, d, j);
        String[] r = ranks.get(d);
        for (Node n : docs.get(d)) {
          long site = Arrays.binarySearch(r, n.site);
          if (k128) {
            id.setAtIndex(JAVA_LONG, 2 * j, n.ts);
            id.setAtIndex(JAVA_LONG, 2 * j + 1, (site << 32) | n.tx);
          } else {
            id.setAtIndex(JAVA_LONG, j, (n.ts << (siteBits + txBits)) | (site << txBits) | n.tx);
          }
          long c0 = CW_NIL, c1 = CW_NIL;
          if (n.causeKind == 0) {
            long cs = Arrays.binarySearch(r, n.csite);
            if (k128) { c0 = n.cts; c1 = (cs << 32) | n.ctx; }
            else c0 = (n.cts << (siteBits + txBits)) | (cs << txBits) | n.ctx;
          } else if (n.causeKind == 2) {
            c0 = k128 ? CW_NIL : NON_ID_CAUSE;
            c1 = NON_ID_CAUSE;
          }
          if (k128) {
            cause.setAtIndex(JAVA_LONG, 2 * j, c0);
            cause.setAtIndex(JAVA_LONG, 2 * j + 1, c1);
          } else {
            cause.setAtIndex(JAVA_LONG, j, c0);
          }
          kind.set(JAVA_BYTE, j, (byte) n.kind);
          j++;
        }
      }
      off.setAtIndex(JAVA_LONG, D, j);
      MemorySegment perm = a.allocate(JAVA_INT, Math.max(1, N));
      MemorySegment bits = a.allocate(JAVA_INT, Math.max(1, (N + 31) / 32));
      MemorySegment vcount = a.allocate(JAVA_INT, Math.max(1, D));
      MemorySegment maxTs = a.allocate(JAVA_LONG, Math.max(1, D));
      MemorySegment status = a.allocate(JAVA_INT, Math.max(1, D));
      MemorySegment yarn = a.allocate(JAVA_INT, Math.max(1, N));
      MemorySegment res = a.allocate(LIST_RESULT);
      res.set(ADDRESS, 0, perm);
      res.set(ADDRESS, 8, bits);
      res.set(ADDRESS, 16, vcount);
      res.set(ADDRESS, 24, maxTs);
      res.set(ADDRESS, 32, status);
      res.set(ADDRESS, 40, yarn);
      if (k128) {
        MemorySegment b = a.allocate(LIST_BATCH_K128);
        b.set(JAVA_LONG, 0, D);
        b.set(ADDRESS, 8, off);
        b.set(ADDRESS, 16, id);
        b.set(ADDRESS, 24, cause);
        b.set(ADDRESS, 32, kind);
        check((int) WEAVE_LISTS_K128.invokeExact(ctx, b, res, CW_MEM_HOST), "cw_weave_lists_k128");
      } else {
        MemorySegment b = a.allocate(LIST_BATCH);
        b.set(JAVA_LONG, 0, D);
        b.set(ADDRESS, 8, off);
        b.set(ADDRESS, 16, id);
        b.set(ADDRESS, 24, cause);
        b.set(ADDRESS, 32, kind);
        b.set(JAVA_INT, 40, tsBits + siteBits + txBits);  // key_bits
        b.set(JAVA_INT, 44, siteBits + txBits);            // ts_shift
        b.set(JAVA_INT, 48, txBits);                       // site_shift
        b.set(JAVA_INT, 52, siteBits);                     // site_bits (yarns)
        check((int) WEAVE_LISTS.invokeExact(ctx, b, res, CW_MEM_HOST), "cw_weave_lists");
      }
      ListResult[] out = new ListResult[D];
      for (int d = 0; d < D; d++) {
        int lo = (int) off.getAtIndex(JAVA_LONG, d), hi = (int) off.getAtIndex(JAVA_LONG, d + 1);
        ListResult r = new ListResult();
        r.weavePerm = new int[hi - lo];
        r.yarnPerm = new int[hi - lo];
        r.rendered = new boolean[hi - lo];
        for (int g = lo; g < hi; g++) {
          r.weavePerm[g - lo] = perm.getAtIndex(JAVA_INT, g);
          r.yarnPerm[g - lo] = yarn.getAtIndex(JAVA_INT, g);
          r.rendered[g - lo] = ((bits.getAtIndex(JAVA_INT, g >>> 5) >>> (g & 31)) & 1) != 0;
        }
        r.visibleCount = vcount.getAtIndex(JAVA_INT, d);
        r.maxTs = maxTs.getAtIndex(JAVA_LONG, d);
        r.status = status.getAtIndex(JAVA_INT, d);
        out[d] = r;
      }
      return out;
    }
  }

  // ================================================================= maps ====
  /** Results of one map collection: one key weave per key (keys as the
   *  caller's key indices; -1 = the id key / nil key quirk, SURVEY F8c). */
  public static final class MapResult {
    public long[] segKey;      // key token (or CW_MAP_ID_KEY | packed id, or CW_NIL)
    public int[][] keyWeave;   // per key weave: node indices (root = -1 first)
    public int[] active;       // per key weave: active node index, -1 = ::blank
    public int status;
  }

  /** A map id packed as ts | site rank | tx; the root id [0 "0" 0] is 0 whatever
   *  rank "0" has (cause_amd/pack.py pack_maps). */
  static long packMapId(String[] ranks, long ts, String site, long tx, int siteBits, int txBits) {
    if (ts == 0 && tx == 0 && site.equals("0")) return 0L;
    long rank = Arrays.binarySearch(ranks, site);
    return (ts << (siteBits + txBits)) | (rank << txBits) | tx;
  }

  /** c.map/weave 1-arity (map.cljc:21-45) + active-node (:47-59) for a batch of
   *  collections; keyToken[j] = the key token of node j when causeKind is 2. */
  public MapResult[] weaveMaps(List<List<Node>> colls, List<long[]> keyTokens, int tokenBits)
      throws Throwable {
    int D = colls.size();
    long N = 0, mts = 0, mtx = 0;
    int msite = 0;
    List<String[]> ranks = new ArrayList<>(D);
    for (List<Node> d : colls) {
      List<Node> withRoot = new ArrayList<>(d);
      withRoot.add(new Node(0, "0", 0, 1, 0, null, 0, KIND_ROOT));
      String[] r = internSites(withRoot);
      // site-ids may sort before "0" (String.compareTo, e.g. " a ", list_test.cljc:85-96):
      // the virtual root [0 "0" 0] still packs to 0 and so does a cause naming it; an
      // id with ts >= 1 packs above 0 whatever its site's rank.  Only an id (a node's or
      // an id cause) that itself sorts before the root id (ts 0) is refused -- as
      // cause_amd/pack.py does.
      for (Node n : d) {
        if (n.ts == 0 && n.site.compareTo("0") < 0)
          throw new IllegalArgumentException("map node id [0 \"" + n.site + "\" " + n.tx
              + "] sorts before the root id");
        // an id cause [0 s tx] with s before "0" would pack onto the root id
        if (n.causeKind == 0 && n.cts == 0 && n.csite.compareTo("0") < 0)
          throw new IllegalArgumentException("map cause id [0 \"" + n.csite + "\" " + n.ctx
              + "] sorts before the root id");
      }
      ranks.add(r);
      msite = Math.max(msite, r.length - 1);
      for (Node n : d) {
        mts = Math.max(mts, Math.max(n.ts, n.causeKind == 0 ? n.cts : 0));
        mtx = Math.max(mtx, Math.max(n.tx, n.causeKind == 0 ? n.ctx : 0));
      }
      N += d.size();
    }
    int tsBits = bits(mts), siteBits = bits(msite), txBits = bits(mtx);
    if (tsBits + siteBits + txBits > 62) throw new IllegalArgumentException("map ids must fit 62 bits");
    try (Arena a = Arena.ofConfined()) {
      MemorySegment off = a.allocate(JAVA_LONG, D + 1);
      MemorySegment id = a.allocate(JAVA_LONG, Math.max(1, N));
      MemorySegment cause = a.allocate(JAVA_LONG, Math.max(1, N));
      MemorySegment isId = a.allocate(JAVA_BYTE, Math.max(1, N));
      MemorySegment kind = a.allocate(JAVA_BYTE, Math.max(1, N));
      long j = 0;
      for (int d = 0; d < D; d++) {
        off.setAtIndex(JAVA_LONG, d, j);
        String[] r = ranks.get(d);
        long[] tok = keyTokens.get(d);
        int k = 0;
        for (Node n : colls.get(d)) {
          id.setAtIndex(JAVA_LONG, j, packMapId(r, n.ts, n.site, n.tx, siteBits, txBits));
          if (n.causeKind == 0) {
            cause.setAtIndex(JAVA_LONG, j, packMapId(r, n.cts, n.csite, n.ctx, siteBits, txBits));
            isId.set(JAVA_BYTE, j, (byte) 1);
          } else if (n.causeKind == 1) {  // nil: the nil key (cause_is_id = 2)
            cause.setAtIndex(JAVA_LONG, j, 0L);
            isId.set(JAVA_BYTE, j, (byte) 2);
          } else {
            cause.setAtIndex(JAVA_LONG, j, tok[k]);
            isId.set(JAVA_BYTE, j, (byte) 0);
          }
          kind.set(JAVA_BYTE, j, (byte) n.kind);
          j++;
          k++;
        }
      }
      off.setAtIndex(JAVA_LONG, D, j);
      long cap = Math.max(1, N);
      MemorySegment segOff = a.allocate(JAVA_LONG, cap + 1);
      MemorySegment segColl = a.allocate(JAVA_INT, cap);
      MemorySegment segKey = a.allocate(JAVA_LONG, cap);
      MemorySegment segActive = a.allocate(JAVA_LONG, cap);
      MemorySegment segPerm = a.allocate(JAVA_INT, N + cap);
      MemorySegment status = a.allocate(JAVA_INT, Math.max(1, D));
      MemorySegment b = a.allocate(MAP_BATCH);
      b.set(JAVA_LONG, 0, D);
      b.set(ADDRESS, 8, off);
      b.set(ADDRESS, 16, id);
      b.set(ADDRESS, 24, cause);
      b.set(ADDRESS, 32, isId);
      b.set(ADDRESS, 40, kind);
      b.set(JAVA_INT, 48, tsBits + siteBits + txBits);
      b.set(JAVA_INT, 52, tokenBits);
      MemorySegment res = a.allocate(MAP_RESULT);
      res.set(JAVA_LONG, 0, cap);
      res.set(ADDRESS, 16, segOff);
      res.set(ADDRESS, 24, segColl);
      res.set(ADDRESS, 32, segKey);
      res.set(ADDRESS, 40, segActive);
      res.set(ADDRESS, 48, segPerm);
      res.set(ADDRESS, 56, status);
      check((int) WEAVE_MAPS.invokeExact(ctx, b, res, CW_MEM_HOST), "cw_weave_maps");
      int S = (int) res.get(JAVA_LONG, 8);
      MapResult[] out = new MapResult[D];
      int[] perColl = new int[D];
      for (int s = 0; s < S; s++) perColl[segColl.getAtIndex(JAVA_INT, s)]++;
      for (int d = 0; d < D; d++) {
        out[d] = new MapResult();
        out[d].segKey = new long[perColl[d]];
        out[d].keyWeave = new int[perColl[d]][];
        out[d].active = new int[perColl[d]];
        out[d].status = status.getAtIndex(JAVA_INT, d);
      }
      int[] fill = new int[D];
      for (int s = 0; s < S; s++) {
        int d = segColl.getAtIndex(JAVA_INT, s), i = fill[d]++;
        long lo = segOff.getAtIndex(JAVA_LONG, s), hi = segOff.getAtIndex(JAVA_LONG, s + 1);
        int[] kw = new int[(int) (hi - lo)];
        for (long g = lo; g < hi; g++) kw[(int) (g - lo)] = segPerm.getAtIndex(JAVA_INT, g);
        out[d].segKey[i] = segKey.getAtIndex(JAVA_LONG, s);
        out[d].keyWeave[i] = kw;
        out[d].active[i] = (int) segActive.getAtIndex(JAVA_LONG, s);
      }
      return out;
    }
  }
}
