"use strict";
// TEST INFRASTRUCTURE: what SharedSegmentSequence's event objects compute from a Client
// (sequence/src/sequenceDeltaEvent.ts:40-53 over merge-tree/src/sortedSegmentSet.ts:29-84),
// restated so the GPU box -- where the reference cannot travel -- can run a listener's view
// of a GpuClient's events.  Pinned on the reference's own events (tests/test_js_facade.py:
// the same ranges from the fixture's ordinals and positions).
function ordinalOf(item) { return item.segment.ordinal; }

// SortedSegmentSet.findOrdinalPosition / addOrUpdate: kept sorted by ordinal (JS string
// compare), an item whose ordinal is already present is not added (SURVEY Q8)
function addOrUpdate(items, item) {
    const ord = ordinalOf(item);
    if (items.length === 0) { items.push(item); return; }
    let start = 0, end = items.length - 1;
    for (;;) {
        const index = start + Math.floor((end - start) / 2);
        const o = ordinalOf(items[index]);
        if (o > ord) {
            if (start === index) { items.splice(index, 0, item); return; }
            end = index - 1;
        } else if (o < ord) {
            if (index === end) { items.splice(index + 1, 0, item); return; }
            start = index + 1;
        } else {
            return;
        }
    }
}

// SequenceEvent.ranges: {operation, position (Client.getPosition at the call), propertyDeltas, segment}
function sequenceEventRanges(deltaArgs, client) {
    const items = [];
    for (const delta of deltaArgs.deltaSegments) {
        addOrUpdate(items, { operation: deltaArgs.operation, position: client.getPosition(delta.segment),
            propertyDeltas: delta.propertyDeltas, segment: delta.segment });
    }
    return items;
}

module.exports = { sequenceEventRanges };
