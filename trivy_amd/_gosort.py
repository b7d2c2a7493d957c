"""Go 1.19 `sort.Slice` (pdqsort_func) for the analyzer-level AnalysisResult.Sort.

`sort.Slice(x, less)` calls `pdqsort_func(lessSwap{less, swap}, 0, n, bits.Len(n))`
(sort/slice.go, sort/zsortfunc.go, sort/sort.go xorshift).  The algorithm is
unstable, so the order of findings that compare equal under the reference's
`less` (same RuleID and same censored Match, `pkg/fanal/secret/scanner.go:405-410`)
depends on it once a file has more than 12 findings.  Restated from the published
Go 1.19 algorithm; no reference test pins the >12 case (labelled "derived").
"""


class _Data:
    __slots__ = ("x", "less")

    def __init__(self, x, less):
        self.x = x
        self.less = less

    def Less(self, i, j):
        return self.less(self.x[i], self.x[j])

    def Swap(self, i, j):
        x = self.x
        x[i], x[j] = x[j], x[i]


def _bits_len(n):
    return n.bit_length()


def insertion_sort(d, a, b):
    for i in range(a + 1, b):
        j = i
        while j > a and d.Less(j, j - 1):
            d.Swap(j, j - 1)
            j -= 1


def sift_down(d, lo, hi, first):
    root = lo
    while True:
        child = 2 * root + 1
        if child >= hi:
            return
        if child + 1 < hi and d.Less(first + child, first + child + 1):
            child += 1
        if not d.Less(first + root, first + child):
            return
        d.Swap(first + root, first + child)
        root = child


def heap_sort(d, a, b):
    first, lo, hi = a, 0, b - a
    for i in range((hi - 1) // 2, -1, -1):
        sift_down(d, i, hi, first)
    for i in range(hi - 1, -1, -1):
        d.Swap(first, first + i)
        sift_down(d, lo, i, first)


UNKNOWN, INCREASING, DECREASING = 0, 1, 2
_MASK64 = (1 << 64) - 1


def pdqsort(d, a, b, limit):
    max_insertion = 12
    was_balanced = True
    was_partitioned = True
    while True:
        length = b - a
        if length <= max_insertion:
            insertion_sort(d, a, b)
            return
        if limit == 0:
            heap_sort(d, a, b)
            return
        if not was_balanced:
            break_patterns(d, a, b)
            limit -= 1
        pivot, hint = choose_pivot(d, a, b)
        if hint == DECREASING:
            reverse_range(d, a, b)
            pivot = (b - 1) - (pivot - a)
            hint = INCREASING
        if was_balanced and was_partitioned and hint == INCREASING:
            if partial_insertion_sort(d, a, b):
                return
        if a > 0 and not d.Less(a - 1, pivot):
            mid = partition_equal(d, a, b, pivot)
            a = mid
            continue
        mid, already = partition(d, a, b, pivot)
        was_partitioned = already
        left_len, right_len = mid - a, b - mid
        balance_threshold = length // 8
        if left_len < right_len:
            was_balanced = left_len >= balance_threshold
            pdqsort(d, a, mid, limit)
            a = mid + 1
        else:
            was_balanced = right_len >= balance_threshold
            pdqsort(d, mid + 1, b, limit)
            b = mid


def partition(d, a, b, pivot):
    d.Swap(a, pivot)
    i, j = a + 1, b - 1
    while i <= j and d.Less(i, a):
        i += 1
    while i <= j and not d.Less(j, a):
        j -= 1
    if i > j:
        d.Swap(j, a)
        return j, True
    d.Swap(i, j)
    i += 1
    j -= 1
    while True:
        while i <= j and d.Less(i, a):
            i += 1
        while i <= j and not d.Less(j, a):
            j -= 1
        if i > j:
            break
        d.Swap(i, j)
        i += 1
        j -= 1
    d.Swap(j, a)
    return j, False


def partition_equal(d, a, b, pivot):
    d.Swap(a, pivot)
    i, j = a + 1, b - 1
    while True:
        while i <= j and not d.Less(a, i):
            i += 1
        while i <= j and d.Less(a, j):
            j -= 1
        if i > j:
            break
        d.Swap(i, j)
        i += 1
        j -= 1
    return i


def partial_insertion_sort(d, a, b):
    max_steps, shortest_shifting = 5, 50
    i = a + 1
    for _ in range(max_steps):
        while i < b and not d.Less(i, i - 1):
            i += 1
        if i == b:
            return True
        if b - a < shortest_shifting:
            return False
        d.Swap(i, i - 1)
        if i - a >= 2:
            j = i - 1
            while j >= 1:
                if not d.Less(j, j - 1):
                    break
                d.Swap(j, j - 1)
                j -= 1
        if b - i >= 2:
            j = i + 1
            while j < b:
                if not d.Less(j, j - 1):
                    break
                d.Swap(j, j - 1)
                j += 1
    return False


def break_patterns(d, a, b):
    length = b - a
    if length >= 8:
        r = length & _MASK64
        modulus = 1 << _bits_len(length)
        idx = a + (length // 4) * 2 - 1
        for i in range(3):
            r ^= (r << 13) & _MASK64
            r ^= r >> 17
            r ^= (r << 5) & _MASK64
            other = r & (modulus - 1)
            if other >= length:
                other -= length
            d.Swap(idx - 1 + i, a + other)


def choose_pivot(d, a, b):
    shortest_ninther, max_swaps = 50, 4 * 3
    l = b - a
    swaps = [0]
    i = a + l // 4 * 1
    j = a + l // 4 * 2
    k = a + l // 4 * 3
    if l >= 8:
        if l >= shortest_ninther:
            i = median_adjacent(d, i, swaps)
            j = median_adjacent(d, j, swaps)
            k = median_adjacent(d, k, swaps)
        j = median(d, i, j, k, swaps)
    if swaps[0] == 0:
        return j, INCREASING
    if swaps[0] == max_swaps:
        return j, DECREASING
    return j, UNKNOWN


def order2(d, a, b, swaps):
    if d.Less(b, a):
        swaps[0] += 1
        return b, a
    return a, b


def median(d, a, b, c, swaps):
    a, b = order2(d, a, b, swaps)
    b, c = order2(d, b, c, swaps)
    a, b = order2(d, a, b, swaps)
    return b


def median_adjacent(d, a, swaps):
    return median(d, a - 1, a, a + 1, swaps)


def reverse_range(d, a, b):
    i, j = a, b - 1
    while i < j:
        d.Swap(i, j)
        i += 1
        j -= 1


def sort_slice(x, less):
    """In-place Go `sort.Slice(x, less)`; `less(a, b)` compares elements."""
    n = len(x)
    pdqsort(_Data(x, less), 0, n, _bits_len(n))
    return x
