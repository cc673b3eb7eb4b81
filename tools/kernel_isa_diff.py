"""Compare two kernel_isa_dump.py directories: kernels identical by name and
body, kernels renamed with an identical body (a template argument dropped),
kernels only in one build, and kernels whose body changed.

    python tools/kernel_isa_diff.py BEFORE_DIR AFTER_DIR"""
import hashlib
import os
import sys


def load(d):
    out = {}
    for f in sorted(os.listdir(d)):
        out[f[:-2]] = open(os.path.join(d, f)).read()
    return out


def main():
    a, b = load(sys.argv[1]), load(sys.argv[2])
    h = lambda s: hashlib.sha1(s.encode()).hexdigest()  # noqa: E731
    same = [k for k in a if k in b and a[k] == b[k]]
    changed = [k for k in a if k in b and a[k] != b[k]]
    only_a = [k for k in a if k not in b]
    only_b = [k for k in b if k not in a]
    by_body_b = {}
    for k in only_b:
        by_body_b.setdefault(h(b[k]), []).append(k)
    renamed, removed = [], []
    for k in only_a:
        m = by_body_b.get(h(a[k]))
        if m:
            renamed.append((k, m.pop(0)))
        else:
            removed.append(k)
    added = [k for v in by_body_b.values() for k in v]
    print("kernels before %d, after %d" % (len(a), len(b)))
    print("identical (name and every instruction): %d" % len(same))
    print("renamed, identical body: %d" % len(renamed))
    for x, y in renamed:
        print("   %s -> %s" % (x, y))
    print("removed: %d" % len(removed))
    for x in removed:
        print("   %s (%d instructions)" % (x, a[x].count("\n")))
    print("added: %d" % len(added))
    for x in added:
        print("   %s" % x)
    print("changed body: %d" % len(changed))
    for x in changed:
        print("   %s" % x)
    return 1 if (changed or added) else 0


if __name__ == "__main__":
    sys.exit(main())
