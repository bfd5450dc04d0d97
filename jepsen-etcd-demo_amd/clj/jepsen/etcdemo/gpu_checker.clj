(ns jepsen.etcdemo.gpu-checker
  "Batched MI355X linearizability checker for the register workload: a drop-in
  for

    (independent/checker
      (checker/compose
        {:linear   (checker/linearizable {:model (model/cas-register)
                                          :algorithm :linear})
         :timeline (timeline/html)}))

  at src/jepsen/etcdemo.clj:115-119.  The whole history goes to liblincheck.so
  in one native call (lc_pack + lc_check_batch, include/lincheck.h) through
  JNA direct mapping (jepsen.etcdemo.LincheckNative; JNA 4.1.0 is already on
  the demo's classpath, jepsen.etcdemo.iml:61-62).  The result has
  independent/checker's shape:
    {:valid? .. :results {k {:valid? .. :linear {...} :timeline {...}}}
     :failures [k ..]}
  with each :linear map shaped as jepsen.checker/linearizable's: :valid?,
  :analyzer, and for a key that is not valid :op, :previous-ok, :last-op,
  :configs and :final-paths (truncated to 10), rendered natively by
  lc_report -- the same rendering the Python mirror decodes.

  NOT EXERCISED IN THIS REPOSITORY: the build container has no JVM, no
  Clojure and no Leiningen.  The same ABI and the same report decoding are
  exercised from Python (jepsen-etcd-demo_amd/lincheck/, tests/)."
  (:require [clojure.tools.logging :refer [warn]]
            [jepsen [checker :as checker]
                    [independent :as independent]
                    [store :as store]]
            [jepsen.checker.timeline :as timeline]
            [knossos.linear.report :as linear.report]
            [knossos.model :as model])
  (:import (com.sun.jna Memory Pointer)
           (jepsen.etcdemo LincheckNative)))

(defn- check-rc [rc what]
  (when (neg? rc)
    (throw (ex-info (str what " failed: " (LincheckNative/lc_last_error)) {:rc rc})))
  rc)

(def ^:private nil-long Long/MIN_VALUE)  ; LC_NIL / LC_NO_KEY / LC_NO_PROCESS

(def ^:private type-code {:invoke 0 :ok 1 :fail 2 :info 3})
(def ^:private f-code    {:read 0 :write 1 :cas 2 :acquire 4 :release 5 :txn 6})
(def ^:private mop-code  {:read 0 :write 1})    ; LC_MOP_* of a :txn micro-op

;; LC_MODEL_*: which knossos.model the device checks against
(def ^:private model-code {:cas-register 0 :register 1 :mutex 2 :multi-register 3})

;; (model/multi-register) registers named by anything but an integer get ids
;; from 2^62 up (lincheck.history.NAMED_REG_BASE); names holds the reverse map
(def ^:private named-reg-base (bit-shift-left 1 62))
(defn- reg-id [names r]
  (if (integer? r)
    (long r)
    (or (get @names r)
        (let [id (+ named-reg-base (count @names))] (vswap! names assoc r id) id))))

;; LC_ALGO_*: jepsen.checker/linearizable's :algorithm (:linear, :wgl, else
;; competition).  :linear runs knossos.linear's config-set search, :wgl
;; knossos.wgl's own walk (ABI 10), competition :linear and then WGL for the
;; keys :linear gave up on at the budget; lc_result.analyzer (offset 48) says
;; which analysis answered each key.
(defn- algo-code [algorithm] (case algorithm :linear 0 :wgl 1 2))

(def ^:private max-final 10)  ; jepsen.checker/linearizable truncates to 10

(defn- long-or-nil [x] (if (nil? x) nil-long (long x)))

(defn- marshal
  "Writes the history into the struct-of-arrays lc_history (10 x 8 bytes,
  ABI 8).  :txn values go to mop_off / mop; `names` collects named registers."
  [history names]
  (let [n      (count history)
        txns   (keep-indexed (fn [i op]
                               (when (= :txn (:f op))
                                 (let [v (:value op)
                                       v (if (independent/tuple? v) (val v) v)]
                                   (when (seq v) [i v]))))
                             history)
        n-mop  (reduce + 0 (map (comp count second) txns))
        mop-off (when (seq txns) (Memory. (* 8 (inc n))))
        mop    (when (seq txns) (Memory. (max 8 (* 24 n-mop))))
        nbytes (max 8 (* 8 n))
        types  (Memory. (max 1 n))
        fs     (Memory. (max 1 n))
        procs  (Memory. nbytes)
        ks     (Memory. nbytes)
        v0     (Memory. nbytes)
        v1     (Memory. nbytes)
        idx    (Memory. nbytes)
        hist   (Memory. 80)]
    (loop [i 0, ops (seq history)]
      (when ops
        (let [op    (first ops)
              value (:value op)
              [k v] (if (independent/tuple? value) [(key value) (val value)] [nil value])
              fc    (f-code (:f op) 3)
              [a b] (cond (= fc 2) (if (nil? v) [nil nil] v)
                          (<= 4 fc) [nil nil]      ; mutex ops carry no value
                          :else     [v nil])]
          (.setByte types i (byte (type-code (:type op))))
          (.setByte fs i (byte fc))
          (.setLong procs (* 8 i) (if (integer? (:process op)) (long (:process op)) nil-long))
          (.setLong ks (* 8 i) (long-or-nil k))
          (.setLong v0 (* 8 i) (if (= fc 3) nil-long (long-or-nil a)))
          (.setLong v1 (* 8 i) (if (= fc 3) nil-long (long-or-nil b)))
          (.setLong idx (* 8 i) (long (or (:index op) -1)))
          (recur (inc i) (next ops)))))
    (when mop-off
      (let [by-row (into {} txns)]
        (loop [i 0, at 0]
          (.setLong mop-off (* 8 i) at)
          (when (< i n)
            (let [ms (get by-row i)]
              (doseq [[j [f r x]] (map-indexed vector ms)]
                (.setLong mop (* 24 (+ at j)) (long (mop-code f)))
                (.setLong mop (+ 8 (* 24 (+ at j))) (reg-id names r))
                (.setLong mop (+ 16 (* 24 (+ at j))) (long-or-nil x)))
              (recur (inc i) (+ at (count ms))))))))
    (.setLong hist 0 n)
    (doseq [[off m] [[8 types] [16 fs] [24 procs] [32 ks] [40 v0] [48 v1] [56 idx]
                     [64 mop-off] [72 mop]]]
      (.setPointer hist off m))
    {:hist hist :held [types fs procs ks v0 v1 idx mop-off mop]}))

;; One lc_ctx per (device(s), budget, algorithm), created on first use and
;; kept: a context owns its streams, scratch and staging buffers, so repeated
;; checks allocate nothing once their sizes have been seen.  Calls on one
;; context are serialised inside the library.
(defonce ^:private contexts (atom {}))

(defn- lc-create ^Pointer [devices budget algorithm]
  (let [opts (Memory. 224)      ; sizeof(lc_opts), ABI 6
        out  (Memory. 8)
        devs (vec devices)]
    (.clear opts)
    (.setInt opts 0 (int (first devs)))             ; device
    (.setInt opts 4 (int (algo-code algorithm)))    ; algorithm
    (.setLong opts 8 (long budget))                 ; max_configs
    (.setInt opts 16 (int max-final))               ; max_final
    (when (< 1 (count devs))                        ; one key shard per device
      (.setInt opts 36 (int (count devs)))          ; n_devices
      (doseq [[g d] (map-indexed vector devs)]
        (.setInt opts (+ 40 (* 4 g)) (int d))))     ; devices[g]
    (check-rc (LincheckNative/lc_create opts out) "lc_create")
    (.getPointer out 0)))

(defn- context ^Pointer [devices budget algorithm]
  (let [k [(vec devices) budget algorithm]]
    (or (get @contexts k)
        (locking contexts
          (or (get @contexts k)
              (let [ctx (lc-create devices budget algorithm)]
                (swap! contexts assoc k ctx)
                ctx))))))

(defn close!
  "Destroys every cached device context (e.g. at the end of a test run)."
  []
  (locking contexts
    (doseq [ctx (vals @contexts)] (LincheckNative/lc_destroy ctx))
    (reset! contexts {})))

(defn- unwrap
  "An op as it appears in its key's sub-history (independent/subhistory
  unwraps the tuple value)."
  [op]
  (let [v (:value op)]
    (if (independent/tuple? v) (assoc op :value (val v)) op)))

(defn- model-of
  "The knossos model record holding register value x (LC_NIL = nil); for
  multi-register, x is a state id and the map comes from lc_packed_state_map."
  [model x packed i names]
  (let [v (when-not (= x nil-long) x)]
    (case model
      :cas-register (model/cas-register v)
      :register     (model/register v)
      :mutex        (assoc (model/mutex) :locked (= 1 v))
      :multi-register
      (let [n-regs (LincheckNative/lc_packed_state_map packed i (int x) nil nil 0)
            regs   (long-array (max 1 n-regs))
            xs     (long-array (max 1 n-regs))
            by-id  (into {} (map (fn [[r id]] [id r]) names))]
        (check-rc (LincheckNative/lc_packed_state_map packed i (int x) regs xs n-regs) "lc_packed_state_map")
        (model/multi-register
          (into {} (for [j (range n-regs)]
                     [(get by-id (aget regs j) (aget regs j))
                      (let [y (aget xs j)] (when-not (= y nil-long) y))])))))))

(defn- report
  "Decodes lc_report's words for packed key i into the :linear map;
  analyzer is the analysis that answered the key (:linear or :wgl)."
  [history model analyzer packed i valid fail-ev cause ^Memory finals n-final names]
  (let [words (long-array 256)
        fin   (.share finals (* i max-final 16))
        ;; :wgl's :configs are the Wing-Gong frontier at the stuck :ok (lc_report_wgl)
        render (fn [^longs w cap]
                 (if (= analyzer :wgl)
                   (LincheckNative/lc_report_wgl packed i valid fail-ev fin n-final max-final w cap)
                   (LincheckNative/lc_report packed i valid fail-ev fin n-final max-final w cap)))
        need  (check-rc (render words 256) "lc_report")
        words (if (<= need 256)
                words
                (let [w (long-array need)]
                  (check-rc (render w need) "lc_report")
                  w))
        row   (fn [r] (when (<= 0 r) (unwrap (nth history r))))
        op    (fn [inv done]               ; knossos.history/complete's invocation
                (let [o (row inv)
                      d (when (<= 0 done) (:value (row done)))]
                  (cond (and (= :txn (:f o)) (some? d)) (assoc o :value d)  ; a :txn learns its reads
                        (and (nil? (:value o)) (<= 0 done)) (assoc o :value d)
                        :else o)))
        state-model (fn [x] (model-of model x packed i names))
        fail-op (row (aget words 0))
        prev    (row (aget words 1))
        n-cfg   (aget words 2)
        n-paths (aget words 3)
        pos     (volatile! 4)
        take!   (fn [] (let [x (aget words @pos)] (vswap! pos inc) x))
        ops!    (fn [] (vec (repeatedly (take!) #(op (take!) (take!)))))
        configs (vec (repeatedly n-cfg
                                 (fn [] (let [m (state-model (take!))
                                              pending (ops!)
                                              linear  (ops!)]
                                          {:model m :last-op prev :pending pending :linearized linear}))))
        paths   (vec (repeatedly n-paths
                                 (fn []
                                   (let [m0    (state-model (take!))
                                         steps (vec (repeatedly (take!)
                                                                (fn [] (let [o (op (take!) (take!))]
                                                                         {:op o :model (state-model (take!))}))))
                                         bad   (model/step (state-model (take!)) fail-op)]
                                     (into [{:op prev :model m0}]
                                           (conj steps {:op fail-op :model {:msg (:msg bad)}}))))))
        base    {:analyzer analyzer
                 :configs  configs}]
    (case (int valid)
      1 (assoc base :valid? true :final-paths [])
      0 (assoc base :valid? false :op fail-op :previous-ok prev :last-op prev :final-paths paths)
      (cond-> (assoc base :valid? :unknown :final-paths []
                     :cause (nth [:none :nonlin :budget :window :states :error] (long cause) :error))
        fail-op (assoc :op fail-op)))))

(defn check-history
  "Runs the device search over every key; returns {k :linear-map}."
  [history {:keys [device devices budget model algorithm] :as opts
            :or {device 0 budget (bit-shift-left 1 20) model :cas-register
                 algorithm :linear}}]
  (let [history    (vec history)
        names      (volatile! {})                  ; named register -> id
        {:keys [hist held]} (marshal history names)
        init       (when (= model :multi-register) (seq (:init opts)))   ; (model/multi-register init)
        init-mem   (when init (Memory. (* 16 (count init))))
        _          (doseq [[j [r x]] (map-indexed vector init)]
                     (.setLong init-mem (* 16 j) (reg-id names r))
                     (.setLong init-mem (+ 8 (* 16 j)) (long-or-nil x)))
        pack-opts  (doto (Memory. 24) (.clear)                 ; sizeof(lc_pack_opts), ABI 11 (flags 0)
                     (.setInt 0 (int (model-code model)))
                     (.setInt 4 (int (count init)))
                     (.setPointer 8 init-mem))
        out        (Memory. 8)
        _          (check-rc (LincheckNative/lc_pack hist pack-opts out) "lc_pack")
        packed     (.getPointer out 0)]
    (try
      (let [batch    (Memory. 104)               ; sizeof(lc_batch), ABI 8
            _        (check-rc (LincheckNative/lc_packed_view packed batch) "lc_packed_view")
            n-keys   (.getLong batch 0)
            key-ids  (long-array (max 1 n-keys))
            _        (check-rc (LincheckNative/lc_packed_keys packed key-ids) "lc_packed_keys")
            ctx      (context (or devices [device]) budget algorithm)
            n1       (max 1 n-keys)
            valid    (Memory. n1)
            fail-ev  (Memory. (* 4 n1))
            cause    (Memory. n1)
            finals   (Memory. (* 16 max-final n1))
            n-final  (Memory. (* 4 n1))
            analyzer (Memory. n1)
            result   (Memory. 56)]               ; sizeof(lc_result), ABI 10
        (.clear result)
        (.setPointer result 0 valid)
        (.setPointer result 8 fail-ev)
        (.setPointer result 16 cause)
        (.setPointer result 32 finals)
        (.setPointer result 40 n-final)
        (.setPointer result 48 analyzer)
        (check-rc (LincheckNative/lc_check_batch ctx batch result nil) "lc_check_batch")
        (persistent!
          (reduce
            (fn [m i]
              (let [k  (aget key-ids i)
                    v  (.getByte valid i)
                    c  (.getByte cause i)
                    an (if (= 1 (.getByte analyzer i)) :wgl :linear)]
                (assoc! m k
                        (cond
                          ;; the key's sub-history could not be prepared:
                          ;; what check-safe makes of knossos's exception
                          (and (neg? v) (= 5 c))
                          {:valid? :unknown :error (LincheckNative/lc_packed_key_error packed i)}
                          ;; valid keys: no counterexample to render
                          (= 1 v)
                          {:valid? true :analyzer an
                           :configs [] :final-paths []}
                          :else
                          (report history model an packed i v (.getInt fail-ev (* 4 i)) c
                                  finals (.getInt n-final (* 4 i)) @names)))))
            (transient {})
            (range n-keys))))
      (finally
        (LincheckNative/lc_packed_free packed)
        (identity [held init-mem])))))

(defn- render!
  "jepsen.checker/linearizable's counterexample drawing, SURVEY.md 8(f) F-2:
  for a key whose analysis is not valid (`when-not`, so :unknown is not drawn,
  as there), Knossos's own knossos.linear.report/render-analysis! draws the
  decoded analysis -- :op, :previous-ok and :final-paths, the last already
  truncated to 10 -- into linear.svg under the key's store directory.  An
  error while drawing is logged, never raised, as linearizable does."
  [jepsen-test sub lin subdirectory]
  (when-not (:valid? lin)
    (try
      (linear.report/render-analysis!
        sub lin (.getCanonicalPath (store/path! jepsen-test subdirectory "linear.svg")))
      (catch Throwable e
        (warn e "Error rendering linearizability analysis")))))

(defn checker
  "independent/checker over compose{:linear linearizable(cas-register),
  :timeline html}, with the :linear part batched on the GPU.  opts:
  :device (or :devices, a vector: one key shard per entry, checked at once),
  :budget, :model (:cas-register, the default and the demo's; :register,
  :mutex or :multi-register -- with :init, its initial map -- for the other
  Knossos models, SURVEY.md 8(f) F-4) and :algorithm
  (:linear, the demo's; :wgl; anything else = competition)."
  ([] (checker {}))
  ([opts]
   (reify checker/Checker
     (check [_ test history check-opts]
       (let [linear  (check-history history opts)
             tl      (timeline/html)
             results (into {}
                           (for [[k lin] linear]
                             (let [sub (independent/subhistory k history)
                                   dir ["independent" k]
                                   t   (checker/check-safe tl test sub
                                                           (assoc check-opts
                                                                  :subdirectory dir
                                                                  :history-key k))]
                               (render! test sub lin dir)
                               [k {:valid?   (checker/merge-valid [(:valid? lin) (:valid? t)])
                                   :linear   lin
                                   :timeline t}])))]
         {:valid?   (checker/merge-valid (map :valid? (vals results)))
          :results  results
          ;; :unknown is truthy: such keys are not failures (independent/checker)
          :failures (->> results (remove (comp :valid? val)) (map key) vec)})))))
