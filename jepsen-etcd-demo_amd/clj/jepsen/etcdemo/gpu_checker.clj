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
  JNA, which is already on the demo's classpath (jepsen.etcdemo.iml:61-62,
  net.java.dev.jna/jna 4.1.0).  The result has independent/checker's shape:
  {:valid? .. :results {k {:valid? .. :linear {...} :timeline {...}}}
   :failures [k ..]}.

  NOT EXERCISED IN THIS REPOSITORY: the build container has no JVM, no
  Clojure and no Leiningen.  The same ABI is exercised from Python
  (jepsen-etcd-demo_amd/lincheck/_native.py, tests/)."
  (:require [jepsen [checker :as checker]
                    [independent :as independent]]
            [jepsen.checker.timeline :as timeline])
  (:import (com.sun.jna Function Memory NativeLibrary Pointer)
           (com.sun.jna.ptr PointerByReference)))

(def ^:private lib (delay (NativeLibrary/getInstance "lincheck")))

(defn- f ^Function [name] (.getFunction ^NativeLibrary @lib name))

(defn- call-int [name & args]
  (let [rc (.invokeInt (f name) (object-array args))]
    (when (neg? rc)
      (throw (ex-info (str name " failed: "
                           (.invokeString (f "lc_last_error") (object-array []) false))
                      {:rc rc})))
    rc))

(def ^:private nil-long Long/MIN_VALUE)  ; LC_NIL / LC_NO_KEY / LC_NO_PROCESS

(def ^:private type-code {:invoke 0 :ok 1 :fail 2 :info 3})
(def ^:private f-code    {:read 0 :write 1 :cas 2 :acquire 4 :release 5})

;; LC_MODEL_*: which knossos.model the device checks against
(def ^:private model-code {:cas-register 0 :register 1 :mutex 2})

(defn- long-or-nil [x] (if (nil? x) nil-long (long x)))

(defn- marshal
  "Writes the history into the struct-of-arrays lc_history (8 x 8 bytes)."
  [history]
  (let [n      (count history)
        bytes  (max 8 (* 8 n))
        type   (Memory. (max 1 n))
        fn     (Memory. (max 1 n))
        proc   (Memory. bytes)
        key    (Memory. bytes)
        v0     (Memory. bytes)
        v1     (Memory. bytes)
        index  (Memory. bytes)
        hist   (Memory. 64)]
    (doseq [[i op] (map-indexed vector history)]
      (let [value         (:value op)
            [k v]         (if (independent/tuple? value) [(key value) (val value)] [nil value])
            fc            (f-code (:f op) 3)
            [a b]         (cond (= fc 2) (if (nil? v) [nil nil] v)
                                (<= 4 fc) [nil nil]      ; mutex ops carry no value
                                :else     [v nil])]
        (.setByte type i (byte (type-code (:type op))))
        (.setByte fn i (byte fc))
        (.setLong proc (* 8 i) (if (integer? (:process op)) (long (:process op)) nil-long))
        (.setLong key (* 8 i) (long-or-nil k))
        (.setLong v0 (* 8 i) (if (= fc 3) nil-long (long-or-nil a)))
        (.setLong v1 (* 8 i) (if (= fc 3) nil-long (long-or-nil b)))
        (.setLong index (* 8 i) (long (or (:index op) -1)))))
    (.setLong hist 0 n)
    (doseq [[off m] [[8 type] [16 fn] [24 proc] [32 key] [40 v0] [48 v1] [56 index]]]
      (.setPointer hist off m))
    {:hist hist :keep [type fn proc key v0 v1 index]}))

;; LC_ALGO_*: jepsen.checker/linearizable's :algorithm (:linear, :wgl, else
;; competition).  All three run the same device search; only :analyzer differs.
(defn- algo-code [algorithm] (case algorithm :linear 0 :wgl 1 2))

(defn- lc-create [device budget algorithm]
  (let [opts (Memory. 56)
        out  (PointerByReference.)]
    (.clear opts)
    (.setInt opts 0 (int device))
    (.setInt opts 4 (int (algo-code algorithm)))
    (.setLong opts 8 (long budget))
    (.setInt opts 16 (int 10))          ; max_final: jepsen truncates to 10
    (call-int "lc_create" opts out)
    (.getValue out)))

(defn check-history
  "Runs the device search over every key; returns per-key verdict maps."
  [history {:keys [device budget model algorithm]
            :or {device 0 budget (bit-shift-left 1 20) model :cas-register
                 algorithm :linear}}]
  (let [{:keys [hist]} (marshal history)
        pack-opts      (doto (Memory. 4) (.setInt 0 (int (model-code model))))
        packed-ref     (PointerByReference.)
        _              (call-int "lc_pack" hist pack-opts packed-ref)
        packed         (.getValue packed-ref)
        batch          (Memory. 72)
        _              (call-int "lc_packed_view" packed batch)
        n-keys         (.getLong batch 0)
        ctx            (lc-create device budget algorithm)
        valid          (Memory. (max 1 n-keys))
        fail-ev        (Memory. (* 4 (max 1 n-keys)))
        cause          (Memory. (max 1 n-keys))
        result         (Memory. 48)]
    (try
      (.clear result)
      (.setPointer result 0 valid)
      (.setPointer result 8 fail-ev)
      (.setPointer result 16 cause)
      (call-int "lc_check_batch" ctx batch result nil)
      (into {}
            (for [i (range n-keys)]
              (let [k  (.invokeLong (f "lc_packed_key") (object-array [packed (long i)]))
                    v  (.getByte valid i)
                    fe (.getInt fail-ev (* 4 i))
                    op (when (<= 0 fe)
                         (history (.invokeLong (f "lc_packed_event_row")
                                               (object-array [packed (long i) (long fe)]))))]
                [k (cond-> {:valid?   (case v 1 true 0 false :unknown)
                            :analyzer (if (= algorithm :wgl) :wgl :linear)
                            :configs  []
                            :final-paths []}
                     (zero? v) (assoc :op op)
                     (neg? v)  (assoc :cause ([:none :nonlin :budget :window :states :error]
                                              (.getByte cause i))))])))
      (finally
        (.invokeVoid (f "lc_destroy") (object-array [ctx]))
        (.invokeVoid (f "lc_packed_free") (object-array [packed]))))))

(defn checker
  "independent/checker over compose{:linear linearizable(cas-register),
  :timeline html}, with the :linear part batched on the GPU.  opts:
  :device, :budget, :model (:cas-register, the default and the demo's;
  :register or :mutex for the other Knossos models, SURVEY.md 8(f) F-4) and
  :algorithm (:linear, the demo's; :wgl; anything else = competition)."
  ([] (checker {}))
  ([opts]
   (reify checker/Checker
     (check [_ test history check-opts]
       (let [linear (check-history history opts)
             tl     (timeline/html)
             results (into {}
                           (for [[k lin] linear]
                             (let [sub (independent/subhistory k history)
                                   t   (checker/check-safe tl test sub
                                                           (assoc check-opts
                                                                  :subdirectory ["independent" k]
                                                                  :history-key k))]
                               [k {:valid?   (checker/merge-valid [(:valid? lin) (:valid? t)])
                                   :linear   lin
                                   :timeline t}])))]
         {:valid?   (checker/merge-valid (map :valid? (vals results)))
          :results  results
          :failures (->> results (remove (comp :valid? val)) (map key) vec)})))))
