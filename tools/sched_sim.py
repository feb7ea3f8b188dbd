"""Discrete-event model of a pipelined run's schedule (hl_pipeline.h): how
long a run of n pictures takes on P persistent workgroups when every
macroblock task costs about one unit, for a given guaranteed reach R (task
(f+1, x, y) becomes ready once picture f finished reach_task(x+R, y+R)) and
an optional in-task wait for the reach a search actually needs (need >= 0:
the task, once started, also waits for picture f's reach_task(x+need,
y+need)).  Development tool: it prices schedule changes before they are
built.

  python tools/sched_sim.py [pictures] [P] [jitter]
"""
import heapq
import random
import sys

MBW, MBH = 120, 68


def reach_task(X, Y):
    ty = min(Y + 2, MBH - 1)
    k = 3 if ty == MBH - 1 else 2
    return min(X + k, MBW - 1), ty


def simulate(n, P, R, need=-1, jitter=0.0, hop=None, seed=1):
    rng = random.Random(seed)
    hop = 3 * (R + 2) + 6 if hop is None else hop
    nmb = MBW * MBH
    cost = [1.0 + jitter * (rng.random() * 2 - 1) for _ in range(n * nmb)]
    done_t = [None] * (n * nmb)
    # dependency counts
    cnt = [0] * (n * nmb)
    succ = [[] for _ in range(n * nmb)]
    for f in range(n):
        for y in range(MBH):
            for x in range(MBW):
                t = f * nmb + y * MBW + x
                deps = []
                if x > 0:
                    deps.append(t - 1)
                if y > 0:
                    deps.append(f * nmb + (y - 1) * MBW + (x + 1 if x + 1 < MBW else x))
                if f > 0:
                    tx, ty = reach_task(min(x + R, MBW - 1), min(y + R, MBH - 1))
                    deps.append((f - 1) * nmb + ty * MBW + tx)
                cnt[t] = len(deps)
                for d in deps:
                    succ[d].append(t)

    def key(t):
        f, a = divmod(t, nmb)
        y, x = divmod(a, MBW)
        return -((MBW - 1 - x) + 2 * (MBH - 1 - y) - hop * f), f

    ready = [(key(0), 0)]
    events = []  # (time, worker, task)
    free = P
    now = 0.0
    waiting = []  # tasks started but waiting for a reach (time known later): (task, needed task)
    busy_time = 0.0
    while ready or events:
        while free and ready:
            _, t = heapq.heappop(ready)
            free -= 1
            start = now
            if need >= 0 and t >= nmb:
                f, a = divmod(t, nmb)
                y, x = divmod(a, MBW)
                tx, ty = reach_task(min(x + need, MBW - 1), min(y + need, MBH - 1))
                dep = (f - 1) * nmb + ty * MBW + tx
                if done_t[dep] is None:
                    waiting.append((t, dep))
                    continue
            heapq.heappush(events, (start + cost[t], t))
            busy_time += cost[t]
        if not events:
            break
        now, t = heapq.heappop(events)
        done_t[t] = now
        free += 1
        # tasks waiting inside for this one
        still = []
        for (w, dep) in waiting:
            if done_t[dep] is not None:
                heapq.heappush(events, (now + cost[w], w))
                busy_time += cost[w]
            else:
                still.append((w, dep))
        waiting = still
        for s in succ[t]:
            cnt[s] -= 1
            if cnt[s] == 0:
                heapq.heappush(ready, (key(s), s))
    return now, busy_time / (P * now)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    P = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    jit = float(sys.argv[3]) if len(sys.argv) > 3 else 0.3
    work = n * MBW * MBH / P
    print(f"{n} pictures, {P} workgroups, cost jitter +-{jit}: work/P = {work:.1f} units")
    for R, need in ((2, -1), (1, -1), (1, 1), (0, 1), (0, 0)):
        T, util = simulate(n, P, R, need, jit)
        print(f"  R={R} in-task wait for reach {need:>2}: makespan {T:7.1f} units ({T / work:.3f} x work/P), utilisation {util:.3f}")


if __name__ == "__main__":
    main()
