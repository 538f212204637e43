"""Host-side compiler of node labels / taints and pod tolerations / node affinity into the engine's bitmasks
(kg_node_predicates and the kg_pod TaintToleration / NodeAffinity fields, ABI 8), and of node images / pod
containers into the ImageLocality fields (ABI 10, ImageTable).

The Go shim keeps two dense tables per scheduler: the distinct taints (key, value, effect) of the cluster's nodes
and the distinct node-selector predicates the queued pods use — a NodeSelectorRequirement (key, operator, values),
a MatchFields requirement on metadata.name, or one pod.Spec.NodeSelector key=value pair.  Each node row holds
which predicates hold on the node's labels and which taints it carries; each pod holds which taints its
tolerations tolerate and its terms as predicate masks.  The device then evaluates the plugins as bit arithmetic
(koordinator_amd/csrc/defaults_dev.h).

Matching restates upstream semantics (k8s.io/kubernetes v1.24.15, k8s.io/component-helpers v0.24.15 — neither
vendored in the reference):
* Toleration.ToleratesTaint (core/v1/toleration.go): an effect, if set, must equal the taint's; a key, if set, must
  equal the taint's; operator Exists tolerates any value, Equal (or empty) needs the same value.
* nodeaffinity.NodeSelector (component-helpers/scheduling/corev1/nodeaffinity): terms are ORed, requirements of a
  term ANDed, a term with no requirements matches nothing; label operators In / NotIn / Exists / DoesNotExist /
  Gt / Lt (labels.Requirement.Matches: NotIn and DoesNotExist hold when the key is absent, Gt / Lt parse both sides
  as int64 and fail on a parse error); MatchFields only on metadata.name with In / NotIn.
* pod.Spec.NodeSelector: labels.SelectorFromSet — every key present with the same value.
A requirement that does not parse (unknown operator, Gt / Lt without exactly one integer value, a field other than
metadata.name) makes its term fail to match — the lazy-error selector skips such terms — so it compiles to a
predicate that holds on no node.
"""
from __future__ import annotations

import numpy as np

from . import abi

NO_SCHEDULE, PREFER_NO_SCHEDULE, NO_EXECUTE = "NoSchedule", "PreferNoSchedule", "NoExecute"
MAX_IDS = 64


_INT64_MIN, _INT64_MAX = -(1 << 63), (1 << 63) - 1


def _parse_int(s):
    """strconv.ParseInt(s, 10, 64) as labels.Requirement.Matches uses it for Gt / Lt: an optional sign and decimal
    digits only (no underscores, spaces or '0x'), within int64; anything else is a parse error (None)."""
    if not isinstance(s, str) or not s:
        return None
    body = s[1:] if s[0] in "+-" else s
    if not body or not all("0" <= ch <= "9" for ch in body):
        return None
    v = int(s, 10)
    return v if _INT64_MIN <= v <= _INT64_MAX else None


class PredicateTable:
    """The caller's taint and predicate id tables (at most 64 each).  The tables only grow, and a row compiled earlier
    stays right for the ids that existed then: a node row decides the predicates interned before it (predicate_count),
    a pod's tolerated mask the taints interned before it (taint_count, KG_POD_TAINT_TABLE).  The engine refuses a
    schedule call whose queue references a predicate some node row was compiled without, or whose node rows carry a
    taint some pod was compiled without (ABI 11): re-send the node rows / re-stage the pods after the table grows."""

    def __init__(self):
        self.taints: list[tuple] = []
        self.preds: list[tuple] = []
        self.zones: list[str] = []  # (ABI 12) topology.kubernetes.io/zone values, for PodTopologySpread zone keys
        self._taint_id: dict = {}
        self._pred_id: dict = {}

    # ---- interning ----
    def taint_id(self, key: str, value: str, effect: str) -> int:
        t = (key, value or "", effect)
        if t not in self._taint_id:
            if len(self.taints) == MAX_IDS:
                raise OverflowError("more than 64 distinct taints: the pods stay on the Go path")
            self._taint_id[t] = len(self.taints)
            self.taints.append(t)
        return self._taint_id[t]

    def pred_id(self, kind: str, key: str, op: str, values=()) -> int:
        p = (kind, key, op, tuple(values or ()))
        if p not in self._pred_id:
            if len(self.preds) == MAX_IDS:
                raise OverflowError("more than 64 distinct node-selector predicates: the pods stay on the Go path")
            self._pred_id[p] = len(self.preds)
            self.preds.append(p)
        return self._pred_id[p]

    # ---- predicate evaluation (per node update) ----
    @staticmethod
    def _holds(pred, labels: dict, name: str) -> bool:
        kind, key, op, values = pred
        if kind == "field":
            if key != "metadata.name" or op not in ("In", "NotIn"):
                return False
            return (name in values) == (op == "In")
        has = key in labels
        v = labels.get(key)
        if op == "In":
            return has and v in values
        if op == "NotIn":
            return not has or v not in values
        if op == "Exists":
            return has
        if op == "DoesNotExist":
            return not has
        if op in ("Gt", "Lt"):
            if not has or len(values) != 1:
                return False
            a, b = _parse_int(v), _parse_int(values[0])
            if a is None or b is None:
                return False
            return a > b if op == "Gt" else a < b
        return False  # unknown operator: the term never matches

    def node_row(self, labels: dict | None = None, taints: list | None = None, name: str = "") -> np.ndarray:
        """kg_node_predicates of one node: labels {key: value}, taints [{key, value, effect}]."""
        labels = labels or {}
        r = np.zeros(1, dtype=abi.NODE_PRED_DTYPE)
        m = 0
        for k, pr in enumerate(self.preds):
            if self._holds(pr, labels, name):
                m |= 1 << k
        hard = soft = 0
        for t in taints or ():
            eff = t["effect"]
            bit = 1 << self.taint_id(t["key"], t.get("value", ""), eff)
            if eff == PREFER_NO_SCHEDULE:
                soft |= bit
            elif eff in (NO_SCHEDULE, NO_EXECUTE):
                hard |= bit
        r["predicates"], r["taints_hard"], r["taints_soft"] = m, hard, soft
        r["predicate_count"] = len(self.preds)  # ABI 11: predicates interned later are undecided on this row
        z = labels.get(ZONE)
        if z is not None:  # (ABI 12) the node's zone domain, 1-based (0 = no zone label)
            if z not in self.zones:
                if len(self.zones) == abi.MAX_ZONES:
                    raise OverflowError(f"more than {abi.MAX_ZONES} zones: zone spread stays on the Go path")
                self.zones.append(z)
            r["zone"] = self.zones.index(z) + 1
        return r

    # ---- pods (per staging: evaluated against the taints interned so far) ----
    @staticmethod
    def tolerates(tol: dict, taint: tuple) -> bool:
        key, value, effect = taint
        if tol.get("effect") and tol["effect"] != effect:
            return False
        if tol.get("key") and tol["key"] != key:
            return False
        op = tol.get("operator") or "Equal"
        if op == "Exists":
            return True
        if op == "Equal":
            return (tol.get("value") or "") == value
        return False

    def _term_mask(self, term: dict) -> int:
        m = 0
        for req in term.get("matchExpressions") or ():
            m |= 1 << self.pred_id("label", req["key"], req["operator"], req.get("values"))
        for req in term.get("matchFields") or ():
            m |= 1 << self.pred_id("field", req["key"], req["operator"], req.get("values"))
        return m

    def fill_pod(self, pod: np.ndarray, tolerations=None, node_selector: dict | None = None,
                 required_terms: list | None = None, preferred: list | None = None) -> np.ndarray:
        """Fills one kg_pod row's TaintToleration / NodeAffinity fields (in place; returns it).
        required_terms: the NodeSelectorTerms of requiredDuringScheduling (None = not set; [] = set with no terms,
        which matches no node); preferred: [(weight, term)]."""
        row = pod[0] if pod.shape else pod
        tols = list(tolerations or ())
        flags = int(row["flags"]) & ~abi.POD_TAINT_TABLE
        if any(not t.get("key") and t.get("operator") == "Exists" and not t.get("effect") for t in tols):
            tol = (1 << 64) - 1  # tolerates every taint, including ones interned later
        else:
            tol = 0
            for t_id, taint in enumerate(self.taints):
                if any(self.tolerates(t, taint) for t in tols):
                    tol |= 1 << t_id
            if tols:  # decided for the taints interned so far only (ABI 11: the engine checks it against node rows)
                flags |= abi.POD_TAINT_TABLE
                row["taint_count"] = len(self.taints)
        row["flags"] = flags
        sel = 0
        for k, v in (node_selector or {}).items():
            sel |= 1 << self.pred_id("label", k, "In", (v,))
        row["tolerated_taints"] = tol
        row["node_selector"] = sel
        if required_terms is not None:
            if len(required_terms) > abi.MAX_AFF_TERMS:
                raise OverflowError("more than 4 required terms: the pod stays on the Go path")
            terms = [self._term_mask(t) for t in required_terms] or [0]  # no terms: one never-matching term
            row["n_required_terms"] = len(terms)
            row["required_terms"][:] = 0
            row["required_terms"][:len(terms)] = terms
        pref = preferred or []
        if len(pref) > abi.MAX_AFF_TERMS:
            raise OverflowError("more than 4 preferred terms: the pod stays on the Go path")
        row["n_preferred_terms"] = len(pref)
        row["preferred_terms"][:] = 0
        row["preferred_weights"][:] = 0
        for k, (w, term) in enumerate(pref):
            row["preferred_terms"][k] = self._term_mask(term)
            row["preferred_weights"][k] = w
        return pod

    # ---- (ABI 12) reservation affinity (matchReservation, reservation/transformer.go:348-372) ----
    def reservation_predicates(self, node_labels: dict | None, reservation_labels: dict | None,
                               reservation_name: str = "") -> int:
        """kg_node_reservations.predicates of one slot: the predicate bits over matchReservation's fakeNode — named
        after the reservation, the node's labels overlaid with the reservation's.  Like node rows, a slot decides the
        predicates interned before it: intern the queue's reservation affinities first, set the row's
        predicate_count to len(self.preds), and re-send the slots after the table grows (the engine refuses a queue
        using a later predicate)."""
        labels = dict(node_labels or {})
        labels.update(reservation_labels or {})
        m = 0
        for k, pr in enumerate(self.preds):
            if self._holds(pr, labels, reservation_name):
                m |= 1 << k
        return m

    def fill_reservation_affinity(self, pod: np.ndarray, selector: dict | None = None,
                                  required_terms: list | None = None) -> np.ndarray:
        """The pod's required reservation affinity (apiext.ReservationAffinity; GetRequiredReservationAffinity,
        pkg/util/reservation/reservation.go:450-474): reservationSelector {key: value} and the
        ReservationSelectorTerms of requiredDuringScheduling (None = not set; [] = set with no terms, matching
        nothing).  Neither set: no affinity.  Sets KG_POD_RSV_AFFINITY when either is (in place; returns it)."""
        row = pod[0] if pod.shape else pod
        sel = 0
        for k, v in (selector or {}).items():
            sel |= 1 << self.pred_id("label", k, "In", (v,))
        row["reservation_selector"] = sel
        row["n_reservation_terms"] = 0
        row["reservation_terms"][:] = 0
        if required_terms is not None:
            if len(required_terms) > abi.MAX_AFF_TERMS:
                raise OverflowError("more than 4 reservation affinity terms: the pod stays on the Go path")
            terms = [self._term_mask(t) for t in required_terms] or [0]
            row["n_reservation_terms"] = len(terms)
            row["reservation_terms"][:len(terms)] = terms
        flags = int(row["reservation_flags"]) & ~abi.POD_RSV_AFFINITY
        if selector or required_terms is not None:
            flags |= abi.POD_RSV_AFFINITY
        row["reservation_flags"] = flags
        return pod


def normalized_image_name(name: str) -> str:
    """imagelocality normalizedImageName (v1.24.15): no tag after the last '/' → ':latest' appended."""
    return name if name.rfind(":") > name.rfind("/") else name + ":latest"


class ImageTable:
    """The caller's ImageLocality view.  The scheduler cache keeps, per image name of any node's status, the size first
    recorded and the set of nodes listing it (cache.addNodeImageStates); a node's ImageStates holds the names its own
    status lists.  Bits go to the images the queued pods use and some node holds (at most 64); scaledImageScore =
    int64(float64(size) * float64(numNodes) / float64(totalNumNodes)) is the same on every node, so it travels with
    the pod and the device only tests node bits."""

    def __init__(self, node_images: list):
        """node_images[i]: node i's status images as [(names, size_bytes)], in snapshot order."""
        self.total = len(node_images)
        self.size: dict = {}
        self.nodes: dict = {}
        self.node_names = []
        for i, imgs in enumerate(node_images):
            names = set()
            for img_names, size in imgs or ():
                for nm in img_names:
                    if nm not in self.size:
                        self.size[nm] = int(size)
                        self.nodes[nm] = set()
                    self.nodes[nm].add(i)
                    names.add(nm)
            self.node_names.append(names)
        self.bits: dict = {}

    def scaled(self, name: str) -> int:
        spread = float(len(self.nodes[name])) / float(self.total)
        return int(float(self.size[name]) * spread)

    def fill_pod(self, pod: np.ndarray, containers: list) -> np.ndarray:
        """The pod's ImageLocality fields from its container images (in place; returns it)."""
        row = pod[0] if pod.shape else pod
        if len(containers) > abi.MAX_CONTAINERS:
            raise OverflowError("more than 8 containers: the pod stays on the Go path")
        row["n_containers"] = len(containers)
        row["container_image_bit"][:] = -1
        row["container_image_score"][:] = 0
        for c, image in enumerate(containers):
            nm = normalized_image_name(image)
            if nm not in self.size:
                continue  # no node lists it: never in an ImageStates map
            if nm not in self.bits:
                if len(self.bits) == MAX_IDS:
                    raise OverflowError("more than 64 distinct pod images: the pods stay on the Go path")
                self.bits[nm] = len(self.bits)
            row["container_image_bit"][c] = self.bits[nm]
            row["container_image_score"][c] = self.scaled(nm)
        return pod

    def image_count(self) -> int:
        """kg_node_predicates.image_count of a row whose mask node_mask() computes now (ABI 11)."""
        return len(self.bits)

    def node_mask(self, i: int) -> int:
        """kg_node_predicates.images of node i over the bits assigned so far (decided for ids < image_count())."""
        m = 0
        for nm, b in self.bits.items():
            if nm in self.node_names[i]:
                m |= 1 << b
        return m


# ---- (ABI 12) PodTopologySpread / InterPodAffinity match groups ---------------------------------------------------
def selector_matches(selector: dict | None, labels: dict) -> bool:
    """metav1.LabelSelectorAsSelector(selector).Matches(labels): nil matches nothing, {} everything; matchLabels and
    matchExpressions (In / NotIn / Exists / DoesNotExist) are ANDed."""
    if selector is None:
        return False
    for k, v in (selector.get("matchLabels") or {}).items():
        if labels.get(k) != v:
            return False
    for e in selector.get("matchExpressions") or ():
        key, op, values = e["key"], e["operator"], tuple(e.get("values") or ())
        has = key in labels
        if op == "In" and not (has and labels[key] in values):
            return False
        if op == "NotIn" and has and labels[key] in values:
            return False
        if op == "Exists" and not has:
            return False
        if op == "DoesNotExist" and has:
            return False
        if op not in ("In", "NotIn", "Exists", "DoesNotExist"):
            return False
    return True


HOSTNAME = "kubernetes.io/hostname"
ZONE = "topology.kubernetes.io/zone"


class PodGroupTable:
    """The caller's match groups (≤ KG_MAX_MATCH_GROUPS): a label selector with its namespace set — a topology spread
    constraint's selector in the pod's namespace (podtopologyspread/common.go countPodsMatchSelector), a pod-affinity
    term's selector and namespaces (AffinityTerm.Matches; an empty namespace list means the term owner's namespace),
    or the conjunction of a pod's required pod-affinity terms (updateWithAffinityTerms counts a pod only when it matches
    all of them).  Register every group the cluster's pods and the queue use before filling pod rows: a row's
    match_groups covers the groups registered when it was filled.  Accelerated topology keys: kubernetes.io/hostname
    and topology.kubernetes.io/zone for both plugins (the node's zone comes from PredicateTable.node_row); another
    key raises NotImplementedError: the pod stays on the Go path."""

    def __init__(self):
        self.groups: list[tuple] = []  # (kind, payload): ("sel", (selector_repr, namespaces)) / ("and", (gid, ...))
        self._id: dict = {}
        self._sel: list = []

    def _intern(self, key, payload) -> int:
        if key not in self._id:
            if len(self.groups) == abi.MAX_MATCH_GROUPS:
                raise OverflowError(f"more than {abi.MAX_MATCH_GROUPS} match groups: the pods stay on the Go path")
            self._id[key] = len(self.groups)
            self.groups.append(key)
            self._sel.append(payload)
        return self._id[key] + 1

    def group(self, selector: dict | None, namespaces) -> int:
        ns = frozenset(namespaces)
        return self._intern(("sel", repr(selector), ns), ("sel", selector, ns))

    def conjunction(self, gids) -> int:
        gids = tuple(sorted(set(gids)))
        return gids[0] if len(gids) == 1 else self._intern(("and", gids), ("and", gids, None))

    def matches(self, gid: int, labels: dict, namespace: str) -> bool:
        kind, a, b = self._sel[gid - 1]
        if kind == "and":
            return all(self.matches(g, labels, namespace) for g in a)
        return namespace in b and selector_matches(a, labels)

    def match_mask(self, labels: dict, namespace: str) -> int:
        return sum(1 << (g - 1) for g in range(1, len(self.groups) + 1) if self.matches(g, labels, namespace))

    def _term(self, t: dict, namespace: str) -> tuple[int, bool]:
        """(group id, zone-keyed) of one pod (anti-)affinity term."""
        key = t.get("topologyKey", HOSTNAME)
        if key not in (HOSTNAME, ZONE):
            raise NotImplementedError(f"pod affinity topologyKey {key}: hostname and zone are accelerated")
        return self.group(t.get("labelSelector"), t.get("namespaces") or (namespace,)), key == ZONE

    @staticmethod
    def _mask(terms, zone: bool) -> int:
        return sum(1 << (g - 1) for g in {g for g, z in terms if z == zone})

    def fill_pod(self, pod: np.ndarray, labels: dict, namespace: str, spread=(), required_affinity=(),
                 required_anti_affinity=(), preferred_affinity=(), preferred_anti_affinity=(),
                 system_default_selector=None) -> np.ndarray:
        """The ABI 12 fields of one pod.  spread: [{maxSkew, whenUnsatisfiable, labelSelector, topologyKey}] with
        topologyKey kubernetes.io/hostname (default) or topology.kubernetes.io/zone; required_*: [{labelSelector,
        namespaces, topologyKey}] (hostname or zone); preferred_*: [{weight, podAffinityTerm}].
        (ABI 13) system_default_selector: a pod without constraints of its own, under a PodTopologySpread configured
        with the system defaults (defaultingType System), gets them here — hostname maxSkew 3 + zone maxSkew 5,
        ScheduleAnyway, on its owners' selector (buildDefaultConstraints) — flagged KG_SPREAD_SYSTEM_DEFAULT, so scoring
        ignores no node (requireAllTopologies false)."""
        r = pod[0] if pod.ndim else pod
        # buildDefaultConstraints returns no constraints when DefaultSelector is empty (selector.Empty(): a pod
        # without owners — no matchLabels, no matchExpressions)
        sel = system_default_selector
        empty = sel is not None and not (sel.get("matchLabels") or sel.get("matchExpressions") or
                                         {k: v for k, v in sel.items() if k not in ("matchLabels", "matchExpressions")})
        if not spread and sel is not None and not empty:
            spread = [dict(maxSkew=3, whenUnsatisfiable="ScheduleAnyway", labelSelector=system_default_selector,
                           topologyKey=HOSTNAME, _system=True),
                      dict(maxSkew=5, whenUnsatisfiable="ScheduleAnyway", labelSelector=system_default_selector,
                           topologyKey=ZONE, _system=True)]
        if len(spread) > abi.MAX_SPREAD:
            raise NotImplementedError(f"more than {abi.MAX_SPREAD} topology spread constraints")
        seen = set()
        r["n_spread"] = len(spread)
        for c, cons in enumerate(spread):
            key = cons.get("topologyKey", HOSTNAME)
            if key not in (HOSTNAME, ZONE):
                raise NotImplementedError(f"topology spread key {key}: hostname and zone are accelerated")
            hard = cons.get("whenUnsatisfiable", "DoNotSchedule") == "DoNotSchedule"
            if (key, hard) in seen:
                raise ValueError("duplicate {topologyKey, whenUnsatisfiable} spread constraints")
            seen.add((key, hard))
            r["spread_group"][c] = self.group(cons.get("labelSelector"), (namespace,))
            r["spread_max_skew"][c] = cons["maxSkew"]
            r["spread_flags"][c] = ((abi.SPREAD_HARD if hard else 0) | (abi.SPREAD_ZONE if key == ZONE else 0) |
                                    (abi.SPREAD_SYSTEM_DEFAULT if cons.get("_system") else 0))
        terms = [self._term(t, namespace) for t in required_affinity]
        if len(set(terms)) != len(terms):
            # (r5) the ABI carries required terms as a group bitmask; upstream processExistingPod adds
            # HardPodAffinityWeight once per term, so two terms with the same selector, namespaces and key would score
            # differently: such a pod stays on the Go path
            raise NotImplementedError("two required pod-affinity terms with the same selector, namespaces and key")
        r["pod_affinity_terms"] = self._mask(terms, False)
        r["pod_affinity_terms_zone"] = self._mask(terms, True)
        r["pod_affinity_group"] = self.conjunction([g for g, _ in terms]) if terms else 0
        anti = [self._term(t, namespace) for t in required_anti_affinity]
        r["pod_anti_affinity"] = self._mask(anti, False)
        r["pod_anti_affinity_zone"] = self._mask(anti, True)
        pref = [(self._term(t["podAffinityTerm"], namespace), t["weight"]) for t in preferred_affinity]
        pref += [(self._term(t["podAffinityTerm"], namespace), -t["weight"]) for t in preferred_anti_affinity]
        if len(pref) > abi.MAX_POD_PREFERRED:
            raise NotImplementedError(f"more than {abi.MAX_POD_PREFERRED} preferred pod affinity terms")
        r["n_pod_preferred"] = len(pref)
        r["pod_preferred_zone"] = sum(1 << t for t, ((_, z), _) in enumerate(pref) if z)
        for t, ((g, _), w) in enumerate(pref):
            r["pod_preferred_group"][t], r["pod_preferred_weight"][t] = g, w
        r["match_groups"] = self.match_mask(labels, namespace)
        return pod
