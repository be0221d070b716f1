"""eval/eval_dvpq.py ``vpq_eval`` — numpy restatement (test infrastructure only).

Follows eval/eval_dvpq.py:25-101, including its integer semantics: ids arrive as
int32 arrays (eval() builds them with astype(np.int32), :113,124), so the
``ign_id * offset + pred_id`` products in prediction_void_overlap /
prediction_ignored_overlap (:52-62) are evaluated on numpy int32 scalars and wrap.
"""
import numpy as np


def vpq_eval(pred_ids, gt_ids, num_cat=20, max_ins=2 ** 20, ign_id=255, offset=2 ** 30):
    iou = np.zeros(num_cat, np.float64)
    tp = np.zeros(num_cat, np.float64)
    fn = np.zeros(num_cat, np.float64)
    fp = np.zeros(num_cat, np.float64)

    def counts(a):
        u, c = np.unique(a, return_counts=True)
        return dict(zip(u, c))

    pred_areas = counts(pred_ids)
    gt_areas = counts(gt_ids)
    void_id = ign_id * max_ins
    ign_ids = {g for g in gt_areas if (g // max_ins) == ign_id}
    int_areas = counts(gt_ids.astype(np.int64) * offset + pred_ids.astype(np.int64))

    def void_overlap(pid):
        with np.errstate(over="ignore"):
            return int_areas.get(void_id * offset + pid, 0)

    def ignored_overlap(pid):
        tot = 0
        with np.errstate(over="ignore"):
            for g in ign_ids:
                tot += int_areas.get(g * offset + pid, 0)
        return tot

    gt_matched, pred_matched = set(), set()
    for iid, area in int_areas.items():
        gid = int(iid // offset)
        pid = int(iid % offset)
        gcat, pcat = gid // max_ins, pid // max_ins
        if gcat != pcat:
            continue
        union = gt_areas[gid] + pred_areas[pid] - area - void_overlap(pid)
        u = area / union
        if u > 0.5:
            tp[gcat] += 1
            iou[gcat] += u
            gt_matched.add(gid)
            pred_matched.add(pid)
    for gid in gt_areas:
        if gid in gt_matched or gid // max_ins == ign_id:
            continue
        fn[gid // max_ins] += 1
    for pid in pred_areas:
        if pid in pred_matched:
            continue
        if ignored_overlap(pid) / pred_areas[pid] > 0.5:
            continue
        fp[pid // max_ins] += 1
    return iou, tp, fn, fp
