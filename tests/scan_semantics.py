"""Test-side restatement of the reference's range scan over exported leaf slot arrays, for
tables too large for the oracle (BASELINE configs[3] at 100M rows).  Inputs are the host
mirror's leaves in key order (Table.export_leaves: record_count, meta word and the 8 key bytes
per slot) and its router (Table.traverse, == BTree::TraverseToLeaf).

RangeScanBySize (b_tree.cpp:1261-1315): slots in SLOT order, visible records with
KeyCompare(start, key) <= 0 are collected until more than to_scan are held, then sorted --
so in a leaf with unsorted slots a scan can skip keys that sit behind the cut.
Iterator::GetNext (b_tree.h:899-941): pops the front; when one record is left, re-traverses
with le_child = false from its key and rescans with the remaining size, dropping the new batch
if it starts with that same key.  8-byte keys only (KeyCompare = unsigned compare of
order_key)."""
import numpy as np

VISIBLE = np.uint64(1 << 62)


def order_key(k):
    """KeyCompare order of 8-byte keys (b_tree.h:114-134: signed-char my_memcmp over the
    little-endian key bytes) as an unsigned integer: bytes ^ 0x80, most significant first."""
    return (np.asarray(k, np.uint64) ^ np.uint64(0x8080808080808080)).byteswap()


class LeafScanner:
    def __init__(self, tab):
        self.tab = tab
        self.rc, _, meta, keyw = tab.export_leaves()
        self.vis = (meta & VISIBLE) != 0
        self.okey = order_key(keyw)
        self.keyw = keyw
        self.nl = self.rc.size

    def range_scan_by_size(self, leaf, ok, to_scan):
        if to_scan == 0 or leaf >= self.nl:
            return []
        n = int(self.rc[leaf])
        q = np.flatnonzero(self.vis[leaf, :n] & (self.okey[leaf, :n] >= ok))[: to_scan + 1]
        return sorted(int(self.okey[leaf, i]) for i in q)

    def scan(self, start_key, scan_size):
        """Keys (little-endian u64) the TableScanExecutor loop returns for one scan."""
        ok = int(order_key(np.uint64(start_key)))
        leaf = int(self.tab.traverse(np.array([start_key], np.uint64))[0])
        batch = self.range_scan_by_size(leaf, ok, scan_size)
        remaining, out = scan_size, []
        while batch and remaining:
            remaining -= 1
            if len(batch) > 1:
                out.append(batch.pop(0))
                continue
            last = batch.pop(0)
            last_key = order_key(np.uint64(last))
            leaf = int(self.tab.traverse(np.array([last_key], np.uint64), le_child=False)[0])
            batch = self.range_scan_by_size(leaf, last, remaining)
            if batch and batch[0] == last:
                batch = []
            out.append(last)
        return order_key(np.array(out, np.uint64))
