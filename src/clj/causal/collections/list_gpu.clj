(ns causal.collections.list-gpu
  "Drop-in weave-fns for CausalList and CausalMap on the MI355X.

  `weave` has the arities and contract of c.list/weave (list.cljc:20-34):
  (weave ct) is the full reweave, one GPU call; (weave ct node) and
  (weave ct node more) are the reference's own incremental weave-node step
  (list.cljc:29-34: O(n) on the host, no marshalling), captured before
  install! rebinds the var -- a single insert never pays for a whole-document
  round trip.  The GPU weave is bit-exact with the fold, so the incremental
  steps continue from it unchanged.  `map-weave` is the same for c.map/weave
  (map.cljc:21-45).  The full reweave never throws for a ::nodes map the
  reference accepts: orphans, non-Lamport and nil causes are rewoven by the
  library's literal fold (exact path).

  Not loaded or run in this repository's image (no JVM); the Python mirror of
  the same calls is cause_amd/causal.py, which the tests run."
  (:require [causal.collections.shared :as s]
            [causal.collections.list :as c.list]
            [causal.collections.map :as c.map]
            [clojure.spec.alpha :as spec])
  (:import (causal.gpu CauseWeave CauseWeave$Node CauseWeave$ListResult CauseWeave$MapResult)
           (java.util.function Supplier)))

;; The reference's weave-fns as loaded, before install! rebinds the vars: the
;; incremental arities (one node, or one tx run) stay on the host.
(defonce ^:private ref-list-weave c.list/weave)
(defonce ^:private ref-map-weave c.map/weave)

;; One context per thread: a cw_ctx is not thread-safe (include/causeweave.h),
;; and swap! may call a weave-fn from several threads at once.
(def ^:private ^ThreadLocal weaver
  (ThreadLocal/withInitial (reify Supplier (get [_] (CauseWeave. 0)))))

(defn- kind-of [v root?]
  (cond root? CauseWeave/KIND_ROOT
        (= v :causal/hide) CauseWeave/KIND_HIDE
        (= v :causal/h.hide) CauseWeave/KIND_HHIDE
        (= v :causal/h.show) CauseWeave/KIND_HSHOW
        :else CauseWeave/KIND_NORMAL))

(defn- id? [x] (and (vector? x) (= 3 (count x)) (string? (second x))))

(defn- ->native
  "A ::nodes entry [id (cause value)] as a CauseWeave$Node."
  [[[ts site tx :as id] body]]
  (let [[cause v] body
        root? (and (= id s/root-id) (nil? cause) (nil? v) (= 2 (count body)))]
    (if (id? cause)
      (let [[cts csite ctx] cause]
        (CauseWeave$Node. ts site tx 0 cts csite ctx (kind-of v root?)))
      (CauseWeave$Node. ts site tx (if (nil? cause) 1 2) 0 nil 0 (kind-of v root?)))))

(defn- check-status [^long st]
  (when (pos? (bit-and st (bit-or CauseWeave/STATUS_DUP CauseWeave/STATUS_INTERNAL
                                  CauseWeave/STATUS_KEY_RANGE)))
    (throw (ex-info "Nodes outside the weave's domain." {:causes #{:weave-domain} :status st}))))

(defn weave-batch
  "Full reweave of many list cts in ONE GPU call.  Returns the cts with
  ::weave, ::yarns and ::lamport-ts rebuilt (s/refresh-caches, shared.cljc:259-266)."
  [cts]
  (let [docs (mapv (comp vec ::s/nodes) cts)
        res (.weaveLists ^CauseWeave (.get weaver) (mapv #(mapv ->native %) docs))]
    (mapv (fn [ct d ^CauseWeave$ListResult r]
            (check-status (.status r))
            (let [nodes (mapv s/new-node d)]
              (assoc ct
                     ::s/weave (mapv nodes (.weavePerm r))
                     ::s/yarns (reduce (fn [y i]
                                         (let [n (nodes i)]
                                           (update y (second (first n)) (fnil conj []) n)))
                                       {} (.yarnPerm r))
                     ::s/lamport-ts (.maxTs r))))
          cts docs res)))

(defn weave
  "c.list/weave (list.cljc:20-34) on the GPU."
  ([causal-tree] (assoc causal-tree ::s/weave (::s/weave (first (weave-batch [causal-tree])))))
  ([causal-tree node] (ref-list-weave causal-tree node nil))
  ([causal-tree node more-consecutive-nodes-in-same-tx]
   (ref-list-weave causal-tree node more-consecutive-nodes-in-same-tx)))

(defn refresh-caches
  "s/refresh-caches with this weave: spin, refresh-ts and the weave from one call."
  [causal-tree]
  (first (weave-batch [causal-tree])))

;; ------------------------------------------------------------------------ maps
(defn map-weave-batch
  "c.map/weave 1-arity (map.cljc:21-45) for many map cts in ONE GPU call."
  [cts]
  (let [docs (mapv (comp vec ::s/nodes) cts)
        tokens (volatile! {})
        tok (fn [k] (or (@tokens k) (let [t (count @tokens)] (vswap! tokens assoc k t) t)))
        natives (mapv (fn [d]
                        (mapv (fn [[[ts site tx] [cause v]]]
                                (if (spec/valid? ::s/id cause)
                                  (let [[cts csite ctx] cause]
                                    (CauseWeave$Node. ts site tx 0 cts csite ctx (kind-of v false)))
                                  (CauseWeave$Node. ts site tx (if (nil? cause) 1 2) 0 nil 0
                                                    (kind-of v false))))
                              d))
                      docs)
        ;; one token per node, aligned with the node order (CauseWeave.weaveMaps reads
        ;; keyToken[j] for node j); id-caused nodes carry 0, which is never read
        key-tokens (mapv (fn [d]
                           (long-array (map (fn [[_ [cause]]]
                                              (if (or (nil? cause) (spec/valid? ::s/id cause))
                                                0
                                                (tok cause)))
                                            d)))
                         docs)
        token-bits (max 1 (- 64 (Long/numberOfLeadingZeros (max 1 (dec (count @tokens))))))
        res (.weaveMaps ^CauseWeave (.get weaver) natives key-tokens (int token-bits))]
    (mapv (fn [ct d ^CauseWeave$MapResult r]
            (check-status (.status r))
            (let [nodes (mapv s/new-node d)
                  node-map (::s/nodes ct)
                  woven (fn [[id cause v]]
                          [id (if (spec/valid? ::s/id cause) cause s/root-id) v])
                  key-of (fn [[_ cause]]
                           (if (spec/valid? ::s/id cause) (first (get node-map cause)) cause))]
              (assoc ct ::s/weave
                     (into {}
                           (map (fn [^ints kw]
                                  (let [ns (mapv nodes (rest kw))]  ; (first kw) is the root
                                    [(key-of (first ns)) (into [s/root-node] (map woven) ns)])))
                           (.keyWeave r)))))
          cts docs res)))

(defn map-weave
  "c.map/weave (map.cljc:21-45) on the GPU."
  ([causal-tree] (first (map-weave-batch [causal-tree])))
  ([causal-tree node] (ref-map-weave causal-tree node nil))
  ([causal-tree node more-nodes] (ref-map-weave causal-tree node more-nodes)))

(defn install!
  "Route CausalList and CausalMap through the GPU: their protocol methods pass
  the `weave` var's value to s/insert, s/append, s/weft and s/merge-trees
  (list.cljc:188-197, map.cljc's extend-type), so rebinding the vars is the
  whole integration."
  []
  (alter-var-root #'c.list/weave (constantly weave))
  (alter-var-root #'c.map/weave (constantly map-weave)))
