"""LinkedListHeap: a doubly linked list whose elements also sit in an array min-heap
(ScalarDistributions/UpgradingDegrading/LinkedListHeap.py:4-191), the structure behind
the greedy letter merging of degrade()/upgrade().

The construction itself runs natively (csrc/host/tv_construct.cpp, class ListHeap);
this module offers the same Python API for code written against the reference.
Tie behaviour is the reference's: an element rises past a parent of equal key, and
sinks only below a strictly smaller child.
"""


class LinkedListHeapElement:
    __slots__ = ("indexInArray", "key", "data", "leftElementInList", "rightElementInList")

    def __init__(self):
        self.indexInArray = None
        self.key = None
        self.data = None
        self.leftElementInList = None
        self.rightElementInList = None


def indexOfLeftChildInArray(i):
    return 2 * i + 1


def indexOfRightChildInArray(i):
    return 2 * i + 2


def indexOfParentInArray(i):
    return (i + 1) // 2 - 1


class LinkedListHeap:
    def __init__(self, keyList=None, dataList=None):
        assert (keyList is None and dataList is None) or len(dataList) == len(keyList)
        self._head = None
        self._tail = None
        self._heapArray = []
        for key, data in zip(keyList or [], dataList or []):
            self.insertAtTail(key, data)

    def __str__(self):
        parts = []
        e = self._head
        while e is not None:
            parts.append("(indexInArray = %s, key = %s, data = %s)" % (e.indexInArray, e.key, e.data))
            e = e.rightElementInList
        return "head -> " + " <-> ".join(parts) + " <- tail"

    def numberOfElements(self):
        return len(self._heapArray)

    def getHeapMin(self):
        return self._heapArray[0]

    def extractHeapMin(self):
        top = self._heapArray[0]
        left, right = top.leftElementInList, top.rightElementInList
        if left is not None:
            left.rightElementInList = right
        if right is not None:
            right.leftElementInList = left
        last = self._heapArray.pop()
        if self._heapArray:
            self._heapArray[0] = last
            last.indexInArray = 0
            self._sink(last)
        return top

    def updateKey(self, element, newKey):
        old = element.key
        element.key = newKey
        if old < newKey:
            self._sink(element)
        elif old > newKey:
            self._rise(element)

    def insertAtTail(self, key, data):
        e = LinkedListHeapElement()
        e.key, e.data = key, data
        e.indexInArray = len(self._heapArray)
        e.leftElementInList = self._tail
        if self._tail is not None:
            self._tail.rightElementInList = e
        self._tail = e
        if self._head is None:
            self._head = e
        self._heapArray.append(e)
        self._rise(e)

    def returnData(self):
        out = []
        e = self._head
        while e is not None:
            out.append(e.data)
            e = e.rightElementInList
        return out

    def _swap(self, a, b):
        a.indexInArray, b.indexInArray = b.indexInArray, a.indexInArray
        self._heapArray[a.indexInArray] = a
        self._heapArray[b.indexInArray] = b

    def _rise(self, e):
        while True:
            p = indexOfParentInArray(e.indexInArray)
            if p < 0 or self._heapArray[p].key < e.key:
                return
            self._swap(e, self._heapArray[p])

    def _sink(self, e):
        n = len(self._heapArray)
        while True:
            best, bestKey = None, e.key
            for c in (indexOfLeftChildInArray(e.indexInArray), indexOfRightChildInArray(e.indexInArray)):
                if c < n and self._heapArray[c].key < bestKey:
                    best, bestKey = self._heapArray[c], self._heapArray[c].key
            if best is None:
                return
            self._swap(e, best)
