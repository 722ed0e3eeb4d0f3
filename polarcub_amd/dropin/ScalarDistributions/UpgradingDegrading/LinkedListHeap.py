"""Drop-in alias of polarcub_amd.heap."""
from polarcub_amd.heap import (LinkedListHeap, LinkedListHeapElement, indexOfLeftChildInArray,  # noqa: F401
                               indexOfParentInArray, indexOfRightChildInArray)
