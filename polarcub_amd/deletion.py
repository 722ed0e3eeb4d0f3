"""Deletion channel: guard bands, channel simulation and the trellis vector distributions.

Reference-compatible surface (same names, argument order and behaviour):

  Guardbands.addDeletionGuardBands / removeDeletionGuardBands / trimZerosAtEdges   Guardbands.py:4-93
  BinaryTrellis.Vertex / Edge / BinaryTrellis                                      VectorDistributions/BinaryTrellis.py:9-306
  BinaryTrellis.buildTrellis_uniformInput_deletion                                 :309-438
  BinaryTrellis.deletionChannelSimulation                                          :441-461
  CollectionOfBinaryTrellises.CollectionOfBinaryTrellises                           VectorDistributions/CollectionOfBinaryTrellises.py:7-103
  CollectionOfBinaryTrellises.buildCollectionOfBinaryTrellises_uniformInput_deletion :106-129

The decoder hot path does not use these Python objects: a collection built by
buildCollectionOfBinaryTrellises_uniformInput_deletion remembers its received
word, and BinaryPolarEncoderDecoder.decode / encodeDecodeSimulation hand the
received words to the HIP kernel (pcub_sc_decode_deletion) whenever the shape
is supported (no guard-band ones, 1 <= n0 <= 3, 1 <= n - n0 <= 6).  The trellis
objects themselves are the VectorDistribution plugin (built lazily, only when a
caller walks them: genie runs, other shapes, direct use).
"""
import math
import random

import numpy as np

from . import vectors


# --------------------------------------------------------------------------- guard bands (Guardbands.py)

def trimZerosAtEdges(receivedWord):
    """The part of receivedWord from its first 1 to its last 1 ([] when it has none)."""
    w = list(receivedWord)
    ones = [i for i, b in enumerate(w) if b == 1]
    return w[ones[0]:ones[-1] + 1] if ones else []


def addDeletionGuardBands(encodedVector, n, n0, xi, numberOfOnesToAddAtBothEndsOfGuardbands=0):
    """Recursively insert floor(2^((1-xi)(n-1))) zeros between the halves (equations (68)-(69)
    of the deletions paper), optionally framing every innermost block with ones."""
    ones = numberOfOnesToAddAtBothEndsOfGuardbands
    if n <= n0:
        return ([1] * ones + list(encodedVector) + [1] * ones) if ones > 0 else encodedVector
    assert len(encodedVector) % 2 == 0
    half = len(encodedVector) // 2
    gap = [0] * math.floor(2 ** ((1 - xi) * (n - 1)))
    return (list(addDeletionGuardBands(encodedVector[:half], n - 1, n0, xi, ones)) + gap
            + list(addDeletionGuardBands(encodedVector[half:], n - 1, n0, xi, ones)))


def removeDeletionGuardBands(receivedWord, n, n0):
    """Trim, halve and recurse until n <= n0; the list of 2^(n-n0) segments."""
    t = trimZerosAtEdges(receivedWord)
    if n <= n0:
        return [t]
    h = len(t) // 2
    return removeDeletionGuardBands(t[:h], n - 1, n0) + removeDeletionGuardBands(t[h:], n - 1, n0)


def deletionChannelSimulation(codeword, p, seed, randomNumberGenerator=None):
    """Delete each symbol independently with probability p (one rng.random() draw per symbol)."""
    if randomNumberGenerator is not None:
        assert seed is None
        rng = randomNumberGenerator
    else:
        rng = random.Random()
        rng.seed(200 if seed is None else seed)
    return [c for c in codeword if not rng.random() < p]


# --------------------------------------------------------------------------- trellis plugin

class Vertex:
    def __init__(self, stateId=-1, verticalPosInLayer=-1, layer=-1, vertexProb=-1.0):
        self.stateId = stateId
        self.verticalPosInLayer = verticalPosInLayer
        self.layer = layer
        self.outgoingEdges = {}
        self.incomingEdges = {}
        self.vertexProb = vertexProb

    def sanityCheck(self):
        assert self.stateId >= 0 and self.verticalPosInLayer >= 0 and self.layer >= 0

    def getKey(self):
        self.sanityCheck()
        return (self.stateId, self.verticalPosInLayer, self.layer)

    def toString(self, printEdges=True):
        s = "* %s: stateId = %s, verticalPosInLayer = %s, layer = %s, vertexProb = %s\n" % (
            self.getKey(), self.stateId, self.verticalPosInLayer, self.layer, self.vertexProb)
        if printEdges:
            s += "  incoming edges (%d):\n" % len(self.incomingEdges)
            s += "".join("    " + e.toString() + "\n" for e in self.incomingEdges.values())
            s += "  outgoing edges (%d):\n" % len(self.outgoingEdges)
            s += "".join("    " + e.toString() + "\n" for e in self.outgoingEdges.values())
        return s

    def __str__(self):
        return self.toString()


class Edge:
    def __init__(self, fromVertex=None, toVertex=None, edgeLabel=-1, edgeProb=-1.0):
        self.fromVertex = fromVertex
        self.toVertex = toVertex
        self.edgeLabel = edgeLabel
        self.edgeProb = edgeProb

    def sanityCheck(self):
        assert self.fromVertex is not None and self.toVertex is not None and self.edgeLabel != -1
        assert self.fromVertex.layer + 1 == self.toVertex.layer
        assert 0.0 <= self.edgeProb <= 1.0

    def getKey(self):
        self.sanityCheck()
        f, t = self.fromVertex, self.toVertex
        return (f.stateId, f.verticalPosInLayer, f.layer, t.stateId, t.verticalPosInLayer, self.edgeLabel)

    def toString(self):
        return "%s --[lbl=%s,p=%s]--> %s" % (self.fromVertex.getKey(), self.edgeLabel, self.edgeProb,
                                             self.toVertex.getKey())

    def __str__(self):
        return self.toString()


class BinaryTrellis(vectors.VectorDistribution):
    """Trellis over `length` binary inputs; verticesInLayer[l] maps vertex keys to vertices in
    insertion order, and every iteration (transforms, normaliser, marginal) follows that
    order, so sums round exactly as the reference's."""

    def __init__(self, length):
        assert length > 0
        self.length = length
        self.layers = length + 1
        self.verticesInLayer = [dict() for _ in range(self.layers)]

    def __len__(self):
        return self.length

    def _vertex(self, stateId, vpos, layer):
        key = (stateId, vpos, layer)
        d = self.verticesInLayer[layer]
        v = d.get(key)
        if v is None:
            v = d[key] = Vertex(stateId, vpos, layer)
        return v

    def setVertexProb(self, vertex_stateId, vertex_verticalPosInLayer, vertex_layer, vertexProb):
        self._vertex(vertex_stateId, vertex_verticalPosInLayer, vertex_layer).vertexProb = vertexProb

    def addToEdgeProb(self, fromVertex_stateId, fromVertex_verticalPosInLayer, fromVertex_layer, toVertex_stateId,
                      toVertex_verticalPosInLayer, toVertex_layer, edgeLabel, probToAdd):
        f = self._vertex(fromVertex_stateId, fromVertex_verticalPosInLayer, fromVertex_layer)
        t = self._vertex(toVertex_stateId, toVertex_verticalPosInLayer, toVertex_layer)
        self.addToEdgeProb_vertexReferences(f, t, edgeLabel, probToAdd)

    def addToEdgeProb_vertexReferences(self, fromVertex, toVertex, edgeLabel, probToAdd):
        key = (fromVertex.stateId, fromVertex.verticalPosInLayer, fromVertex.layer, toVertex.stateId,
               toVertex.verticalPosInLayer, edgeLabel)
        e = fromVertex.outgoingEdges.get(key)
        if e is None:
            assert key not in toVertex.incomingEdges
            e = Edge(fromVertex, toVertex, edgeLabel, 0.0)
            fromVertex.outgoingEdges[key] = e
            toVertex.incomingEdges[key] = e
        e.edgeProb += probToAdd

    def getEdgeProb(self, fromVertex_stateId, fromVertex_verticalPosInLayer, fromVertex_layer, toVertex_stateId,
                    toVertex_verticalPosInLayer, toVertex_layer, edgeLabel):
        f = self.verticesInLayer[fromVertex_layer][(fromVertex_stateId, fromVertex_verticalPosInLayer,
                                                    fromVertex_layer)]
        t = self.verticesInLayer[toVertex_layer][(toVertex_stateId, toVertex_verticalPosInLayer, toVertex_layer)]
        return self.getEdgeProb_vertexReferences(f, t, edgeLabel)

    def getEdgeProb_vertexReferences(self, fromVertex, toVertex, edgeLabel):
        key = Edge(fromVertex, toVertex, edgeLabel).getKey()
        assert key in fromVertex.outgoingEdges and key in toVertex.incomingEdges
        return fromVertex.outgoingEdges[key].edgeProb

    def toString(self):
        s = "The input alphabet size is 2\nThe number of layers is %d\n" % self.layers
        s += "The number of vertices in each layers is: \n"
        s += ", ".join(str(len(d)) for d in self.verticesInLayer) + "\n"
        for l, d in enumerate(self.verticesInLayer):
            s += "For layer %d, these vertices are:\n" % l
            s += "".join(v.toString(printEdges=True) + "\n" for v in d.values())
        return s

    def __str__(self):
        return self.toString()

    def minusTransform(self):
        return self._combine(None)

    def plusTransform(self, decisionVector):
        return self._combine(decisionVector)

    def _combine(self, decisions):
        """Paths u -> w -> v through every odd layer become edges u -> v of the half-length
        trellis carrying p(u->w) * p(w->v); the label is x0 xor x1 (minus) or, for the
        paths whose x0 xor x1 equals the decision of that input pair, x1 (plus)."""
        half = self.length // 2
        out = BinaryTrellis(half)
        if decisions is not None:
            assert len(decisions) == half
        for v in self.verticesInLayer[0].values():
            out.setVertexProb(v.stateId, v.verticalPosInLayer, 0, v.vertexProb)
        for v in self.verticesInLayer[self.length].values():
            out.setVertexProb(v.stateId, v.verticalPosInLayer, half, v.vertexProb)
        for mid in range(1, self.layers, 2):
            j = mid // 2
            for w in self.verticesInLayer[mid].values():
                for ein in w.incomingEdges.values():
                    u = ein.fromVertex
                    for eout in w.outgoingEdges.values():
                        x = 1 if ein.edgeLabel != eout.edgeLabel else 0
                        if decisions is not None:
                            if x != decisions[j]:
                                continue
                            x = eout.edgeLabel
                        t = eout.toVertex
                        out.addToEdgeProb(u.stateId, u.verticalPosInLayer, j, t.stateId, t.verticalPosInLayer,
                                          j + 1, x, ein.edgeProb * eout.edgeProb)
        return out

    def calcMarginalizedProbabilities(self, normalize=True):
        assert len(self) == 1
        terms = [(e.edgeLabel, v.vertexProb * e.edgeProb * e.toVertex.vertexProb)
                 for v in self.verticesInLayer[0].values() for e in v.outgoingEdges.values()]
        s = 1.0
        if normalize:
            s = 0.0
            for _, p in terms:
                s += p
        m = np.zeros(2)
        for x, p in terms:
            m[x] += p / s
        return m

    def calcNormalizationVector(self):
        out = np.zeros(self.length)
        for i in range(self.length):
            acc = np.zeros(2)
            for v in self.verticesInLayer[i].values():
                for e in v.outgoingEdges.values():
                    acc[e.edgeLabel] += e.edgeProb
            out[i] = np.maximum(acc[0], acc[1])
        return out

    def normalize(self, normalization):
        for i in range(self.length):
            t = normalization[i]
            assert t >= 0
            t = 1 if t == 0 else t
            for v in self.verticesInLayer[i].values():
                for e in v.outgoingEdges.values():
                    e.edgeProb /= t

    normalizeDistList = normalize


def buildTrellis_uniformInput_deletion(receivedWord, codewordLength, deletionProb, trimmedZerosAtEdges,
                                       numberOfOnesToAddAtBothEndsOfGuardbands):
    """Single-state trellis of one received segment: vertex (layer l, vpos i) = "l inputs sent,
    i symbols received"; an input either arrives (label = the received symbol,
    prob 0.5 (1 - pd)) or is deleted (both labels, prob 0.5 pd; a deleted 0 at a
    trimmed edge is certain, prob 0.5)."""
    ones = numberOfOnesToAddAtBothEndsOfGuardbands
    m = len(receivedWord)
    L = codewordLength
    tr = BinaryTrellis(L)
    deletions = L + 2 * ones - m
    if ones > 0:
        assert trimmedZerosAtEdges
        for i in range(1 + min(ones, m)):
            tr.setVertexProb(0, i, 0, math.comb(ones, i) * ((1.0 - deletionProb) ** i)
                             * (deletionProb ** (ones - i)))
        for i in range(m, m - min(ones, m) - 1, -1):
            j = m - i
            tr.setVertexProb(0, i, L, math.comb(ones, j) * ((1.0 - deletionProb) ** j)
                             * (deletionProb ** (ones - j)))
    else:
        tr.setVertexProb(0, 0, 0, 1.0)
        tr.setVertexProb(0, m, L, 1.0)
    if trimmedZerosAtEdges:
        assert m == 0 or (receivedWord[0] == 1 and receivedWord[-1] == 1)
    for l in range(L):
        lo = max(0, l + ones - deletions)
        hi = min(l + ones, m)
        for i in range(lo, hi + 1):
            if i < m:
                y = receivedWord[i]
                tr.addToEdgeProb(0, i, l, 0, i + 1, l + 1, y, 0.5 * (1.0 - deletionProb))
            if l + 1 + ones - deletions <= i:
                for x in (0, 1):
                    edge = (not trimmedZerosAtEdges) or x == 1 or 0 < i < m
                    tr.addToEdgeProb(0, i, l, 0, i, l + 1, x, 0.5 * deletionProb if edge else 0.5)
    return tr


class CollectionOfBinaryTrellises(vectors.VectorDistribution):
    """numberOfTrellises independent trellises over consecutive input blocks; the transform
    that halves them to length 1 collapses the collection to a memoryless vector of their
    un-normalised marginals."""

    def __init__(self, length, numberOfTrellises):
        assert length > 0 and numberOfTrellises > 0 and length % numberOfTrellises == 0
        self.length = length
        self.numberOfTrellises = numberOfTrellises
        self.trellisLength = length // numberOfTrellises
        self._trellises = [BinaryTrellis(self.trellisLength) for _ in range(numberOfTrellises)]
        self._lazy = None
        self.deletion_source = None  # (receivedWord, deletionProb, n, n0, ones) when built from a received word

    @property
    def trellises(self):
        if self._lazy is not None:
            word, pd, n, n0, ones = self._lazy
            self._lazy = None
            L = 1 << n0
            self._trellises = [buildTrellis_uniformInput_deletion(s, L, pd, True, ones)
                               for s in removeDeletionGuardBands(word, n, n0)]
        return self._trellises

    @trellises.setter
    def trellises(self, value):
        self._lazy = None
        self._trellises = value

    def __len__(self):
        return self.length

    def __str__(self):
        s = "This collection of Binary trellis contains %d trellises. Each trellis has input length %d. " \
            "These trellises are\n" % (self.numberOfTrellises, self.trellisLength)
        s += "".join("***\n" + t.toString() for t in self.trellises)
        return s + "***\n"

    def minusTransform(self):
        return self._combine(None)

    def plusTransform(self, decisionVector):
        return self._combine(decisionVector)

    def _combine(self, decisions):
        assert self.length % 2 == 0
        T = self.numberOfTrellises
        sub = len(decisions) // T if decisions is not None else 0

        def kid(i, tr):
            return tr.minusTransform() if decisions is None else tr.plusTransform(decisions[i * sub:(i + 1) * sub])

        if self.length // 2 > T:
            out = CollectionOfBinaryTrellises(self.length // 2, T)
            out.trellises = [kid(i, tr) for i, tr in enumerate(self.trellises)]
            return out
        assert self.length // 2 == T
        out = vectors.BinaryMemorylessVectorDistribution(T)
        for i, tr in enumerate(self.trellises):
            m = kid(i, tr).calcMarginalizedProbabilities(normalize=False)
            out.probs[i][0] = m[0]
            out.probs[i][1] = m[1]
        return out

    def calcMarginalizedProbabilities(self):
        # a collection collapses to a memoryless vector before reaching length 1
        assert False

    def calcNormalizationVector(self):
        return [t.calcNormalizationVector() for t in self.trellises]

    def normalize(self, normalization):
        assert len(normalization) == self.numberOfTrellises
        for t, nv in zip(self.trellises, normalization):
            t.normalize(nv)

    normalizeDistList = normalize


def buildCollectionOfBinaryTrellises_uniformInput_deletion(receivedWord, deletionProb, xi, n, n0,
                                                           numberOfOnesToAddAtBothEndsOfGuardbands, verbosity=0):
    """The xy vector distribution of a received word: one trellis per guard-band segment.
    The trellises are built on first use; the decoder reads deletion_source instead."""
    ones = numberOfOnesToAddAtBothEndsOfGuardbands
    coll = CollectionOfBinaryTrellises(2 ** n, 2 ** (n - n0))
    coll._trellises = []
    coll._lazy = (list(receivedWord), float(deletionProb), int(n), int(n0), int(ones))
    coll.deletion_source = coll._lazy
    if verbosity > 0:
        print("trimmed subwords")
        for s in removeDeletionGuardBands(receivedWord, n, n0):
            print(s)
    return coll


def is_deletion_collection(vd):
    return isinstance(vd, CollectionOfBinaryTrellises) and vd.deletion_source is not None
