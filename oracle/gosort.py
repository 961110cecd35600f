"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Restatement of Go 1.22 ``sort.Slice`` = ``pdqsort_func`` (sort/zsortfunc.go),
used by pkg/fanal/secret/scanner.go:452-457.  For n <= 12 it is an insertion
sort (stable); above that the element order of ties follows pdqsort's
deterministic partitioning -- restated here, PARITY UNPINNED (no reference
test has more than 3 findings per file).
"""


class _Data:
    def __init__(self, items, less):
        self.a = items
        self.lessf = less

    def less(self, i, j):
        return self.lessf(self.a[i], self.a[j])

    def swap(self, i, j):
        a = self.a
        a[i], a[j] = a[j], a[i]


def _bits_len(x):
    return x.bit_length()


def _insertion(d, a, b):
    for i in range(a + 1, b):
        j = i
        while j > a and d.less(j, j - 1):
            d.swap(j, j - 1)
            j -= 1


def _sift_down(d, lo, hi, first):
    root = lo
    while True:
        child = 2 * root + 1
        if child >= hi:
            return
        if child + 1 < hi and d.less(first + child, first + child + 1):
            child += 1
        if not d.less(first + root, first + child):
            return
        d.swap(first + root, first + child)
        root = child


def _heap_sort(d, a, b):
    first, lo, hi = a, 0, b - a
    for i in range((hi - 1) // 2, -1, -1):
        _sift_down(d, i, hi, first)
    for i in range(hi - 1, -1, -1):
        d.swap(first, first + i)
        _sift_down(d, lo, i, first)


_MASK64 = (1 << 64) - 1


def _break_patterns(d, a, b):
    length = b - a
    if length >= 8:
        r = length & _MASK64
        modulus = 1 << _bits_len(length)
        idx = a + (length // 4) * 2 - 1
        for i in range(3):
            r ^= (r << 13) & _MASK64
            r ^= r >> 7
            r ^= (r << 17) & _MASK64
            other = r & (modulus - 1)
            if other >= length:
                other -= length
            d.swap(idx - 1 + i, a + other)


INC, DEC, UNK = 1, 2, 0


def _order2(d, a, b, sw):
    if d.less(b, a):
        sw[0] += 1
        return b, a
    return a, b


def _median(d, a, b, c, sw):
    a, b = _order2(d, a, b, sw)
    b, c = _order2(d, b, c, sw)
    a, b = _order2(d, a, b, sw)
    return b


def _median_adjacent(d, a, sw):
    return _median(d, a - 1, a, a + 1, sw)


def _choose_pivot(d, a, b):
    l = b - a
    sw = [0]
    i = a + l // 4 * 1
    j = a + l // 4 * 2
    k = a + l // 4 * 3
    if l >= 8:
        if l >= 50:
            i = _median_adjacent(d, i, sw)
            j = _median_adjacent(d, j, sw)
            k = _median_adjacent(d, k, sw)
        j = _median(d, i, j, k, sw)
    if sw[0] == 0:
        return j, INC
    if sw[0] == 12:
        return j, DEC
    return j, UNK


def _reverse(d, a, b):
    i, j = a, b - 1
    while i < j:
        d.swap(i, j)
        i += 1
        j -= 1


def _partial_insertion(d, a, b):
    i = a + 1
    for _ in range(5):
        while i < b and not d.less(i, i - 1):
            i += 1
        if i == b:
            return True
        if b - a < 50:
            return False
        d.swap(i, i - 1)
        if i - a >= 2:
            j = i - 1
            while j >= 1:
                if not d.less(j, j - 1):
                    break
                d.swap(j, j - 1)
                j -= 1
        if b - i >= 2:
            j = i + 1
            while j < b:
                if not d.less(j, j - 1):
                    break
                d.swap(j, j - 1)
                j += 1
    return False


def _partition_equal(d, a, b, pivot):
    d.swap(a, pivot)
    i, j = a + 1, b - 1
    while True:
        while i <= j and not d.less(a, i):
            i += 1
        while i <= j and d.less(a, j):
            j -= 1
        if i > j:
            break
        d.swap(i, j)
        i += 1
        j -= 1
    return i


def _partition(d, a, b, pivot):
    d.swap(a, pivot)
    i, j = a + 1, b - 1
    while i <= j and d.less(i, a):
        i += 1
    while i <= j and not d.less(j, a):
        j -= 1
    if i > j:
        d.swap(j, a)
        return j, True
    d.swap(i, j)
    i += 1
    j -= 1
    while True:
        while i <= j and d.less(i, a):
            i += 1
        while i <= j and not d.less(j, a):
            j -= 1
        if i > j:
            break
        d.swap(i, j)
        i += 1
        j -= 1
    d.swap(j, a)
    return j, False


def _pdqsort(d, a, b, limit):
    was_balanced, was_partitioned = True, True
    while True:
        length = b - a
        if length <= 12:
            _insertion(d, a, b)
            return
        if limit == 0:
            _heap_sort(d, a, b)
            return
        if not was_balanced:
            _break_patterns(d, a, b)
            limit -= 1
        pivot, hint = _choose_pivot(d, a, b)
        if hint == DEC:
            _reverse(d, a, b)
            pivot = (b - 1) - (pivot - a)
            hint = INC
        if was_balanced and was_partitioned and hint == INC:
            if _partial_insertion(d, a, b):
                return
        if a > 0 and not d.less(a - 1, pivot):
            a = _partition_equal(d, a, b, pivot)
            continue
        mid, already = _partition(d, a, b, pivot)
        was_partitioned = already
        left, right = mid - a, b - mid
        thr = length // 8
        if left < right:
            was_balanced = left >= thr
            _pdqsort(d, a, mid, limit)
            a = mid + 1
        else:
            was_balanced = right >= thr
            _pdqsort(d, mid + 1, b, limit)
            b = mid


def sort_slice(items, less):
    """In-place ``sort.Slice(items, less)`` with ``less(x, y)`` on elements."""
    _pdqsort(_Data(items, less), 0, len(items), _bits_len(len(items)))
    return items
