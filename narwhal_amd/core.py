"""Core-side batching of the primary's message checks.

The reference's ``Core::run`` (primary/src/core.rs:349-411) takes one ``PrimaryMessage`` at a time
from a single tokio task and blocks on its signature check: ``sanitize_header`` (:306-318),
``sanitize_vote`` (:320-336) and ``sanitize_certificate`` (:338-346).  ``CoreBatcher.submit`` takes
the messages that queued up while the GPU was busy and checks them all with a fixed number of GPU
submissions, then applies the verdicts in ARRIVAL order, so the aggregator state and every returned
error are what the serial loop would have produced:

* one SHA-512 submission for every header id and vote digest (``nw_sha512_many``);
* one strict-verify submission for every header and vote signature (``nw_verify_strict_many``);
* ``primary.verify_certificates`` for the certificates (its own SHA-512, strict and
  certificate-batch submissions).

Only the verdict/stake consumers of ``process_vote`` / ``process_certificate`` are mirrored
(``VotesAggregator`` / ``CertificatesAggregator``, primary/src/aggregators.rs); storage, network,
synchronizer and consensus hand-off are out of scope.  Host logic only: every digest
and verdict comes from libnwcrypto.
"""
from __future__ import annotations

import os
from typing import Callable, Dict, Iterable, List, Optional, Sequence, Tuple

from . import _lib
from .primary import (AuthorityReuse, Certificate, Committee, DagError, Header, InvalidHeaderId,
                      InvalidSignature, MalformedHeader, UnknownAuthority, Vote, committee_slots,
                      verify_certificates)


class TooOld(DagError):
    """DagError::TooOld(digest, round) (primary/src/error.rs:58)."""


class UnexpectedVote(DagError):
    """DagError::UnexpectedVote(digest) (primary/src/error.rs:49)."""


class VotesAggregator:
    """primary/src/aggregators.rs:9-45: votes for our own header -> one certificate at quorum."""

    def __init__(self):
        self.weight = 0
        self.votes: List[Tuple[bytes, bytes]] = []
        self.used = set()

    def append(self, vote: Vote, committee: Committee, header: Header) -> Optional[Certificate]:
        if vote.author in self.used:
            raise AuthorityReuse(vote.author.hex())
        self.used.add(vote.author)
        self.votes.append((vote.author, vote.signature))
        self.weight += committee.stake(vote.author)
        if self.weight >= committee.quorum_threshold():
            self.weight = 0   # quorum is reached only once
            return Certificate(header, list(self.votes))
        return None


class CertificatesAggregator:
    """primary/src/aggregators.rs:48-83: certificates of one round -> parents at quorum."""

    def __init__(self):
        self.weight = 0
        self.certificates: List[Certificate] = []
        self.used = set()

    def append(self, certificate: Certificate, committee: Committee) -> Optional[List[Certificate]]:
        origin = certificate.origin()
        if origin in self.used:
            return None
        self.used.add(origin)
        self.certificates.append(certificate)
        self.weight += committee.stake(origin)
        if self.weight >= committee.quorum_threshold():
            # the reference leaves the weight in place (aggregators.rs:78): every later distinct
            # origin of the round re-triggers with the certificates gathered since
            out, self.certificates = self.certificates, []
            return out
        return None


def state_error(m, gc_round: int, current_header: Header) -> Optional[DagError]:
    """The checks of ``Core::sanitize_*`` that read Core's mutable state (gc_round, the current
    header), in the reference's order; they run before any signature check."""
    if isinstance(m, Header):
        if gc_round > m.round:                                       # core.rs:307-310
            return TooOld(m.id.hex(), m.round)
    elif isinstance(m, Vote):
        if current_header.round > m.round:                           # core.rs:321-324
            return TooOld(None, m.round)
        if not (m.id == current_header.id and m.origin == current_header.author
                and m.round == current_header.round):                # core.rs:327-333
            return UnexpectedVote(m.id.hex())
    elif isinstance(m, Certificate):
        if gc_round > m.round():                                     # core.rs:339-342
            return TooOld(None, m.round())
    else:
        raise TypeError("unexpected core message %r" % (m,))          # core.rs:377
    return None


def check_messages(messages: Sequence, committee: Committee, engine=None, zseed: Optional[bytes] = None,
                   cert_base: int = 0, skip: Optional[Sequence[bool]] = None) -> List[Optional[DagError]]:
    """The state-independent rest of the three ``Core::sanitize_*`` checks (Header::verify,
    Vote::verify, Certificate::verify: primary/src/messages.rs:48-67,131-142,189-215) for many
    messages: per message None (Ok) or the DagError the reference returns.  GPU submissions: one
    SHA-512 batch, one strict-verify batch, and verify_certificates' own submissions.  Messages with
    ``skip[i]`` set are not checked (None)."""
    eng = engine or _lib.default_engine()
    n = len(messages)
    out: List[Optional[DagError]] = [None] * n
    hdr, vot, crt = [], [], []
    for i, m in enumerate(messages):
        if skip is not None and skip[i]:
            continue
        if isinstance(m, Header):
            hdr.append(i)
        elif isinstance(m, Vote):
            if committee.stake(m.author) <= 0:                       # Vote::verify, messages.rs:133-136
                out[i] = UnknownAuthority(m.author.hex())
            else:
                vot.append(i)
        elif isinstance(m, Certificate):
            crt.append(i)
        else:
            raise TypeError("unexpected core message %r" % (m,))
    if hdr or vot:
        committee_slots(eng, committee)   # committee keys in the key cache: the comb path
        # digests: header ids (Header::verify :50) and vote digests (Vote::verify :139), one submission
        dig = eng.sha512_many([messages[i].digest_preimage() for i in hdr] +
                              [messages[i].digest_preimage() for i in vot])
        strict_i, strict_msg = [], []
        for k, i in enumerate(hdr):
            h = messages[i]
            if dig[k][:32] != h.id:
                out[i] = InvalidHeaderId()
            elif committee.stake(h.author) <= 0:
                out[i] = UnknownAuthority(h.author.hex())
            elif any(not committee.has_worker(h.author, w) for w in h.payload.values()):
                out[i] = MalformedHeader(h.id.hex())
            else:
                strict_i.append(i)
                strict_msg.append(h.id)
        for k, i in enumerate(vot):
            strict_i.append(i)
            strict_msg.append(dig[len(hdr) + k][:32])
        # every header and vote signature: one strict-verify submission
        if strict_i:
            ok = eng.verify_strict_many(strict_msg, [messages[i].author for i in strict_i],
                                        [messages[i].signature for i in strict_i])
            for i, good in zip(strict_i, ok):
                if not good:
                    out[i] = InvalidSignature()
    if crt:
        if zseed is None:
            zseed = os.urandom(32)
        errs = verify_certificates([messages[i] for i in crt], committee, eng, zseed, cert_base)
        for i, e in zip(crt, errs):
            out[i] = e
    return out


def sanitize_messages(messages: Sequence, committee: Committee, gc_round: int, current_header: Header,
                      engine=None, zseed: Optional[bytes] = None, cert_base: int = 0) -> List[Optional[DagError]]:
    """The three ``Core::sanitize_*`` checks for many messages at once: per message None (Ok) or the
    DagError the reference returns, with the reference's check order per kind."""
    stale = [state_error(m, gc_round, current_header) for m in messages]
    errs = check_messages(messages, committee, engine, zseed, cert_base, skip=[e is not None for e in stale])
    return [s if s is not None else e for s, e in zip(stale, errs)]


class CoreBatcher:
    """The verdict-consuming part of ``Core`` (primary/src/core.rs:24-73) driven in batches.

    ``submit(messages)`` sanitizes a batch and then processes the accepted messages in arrival
    order: a vote goes to the ``VotesAggregator`` of the current header (``process_vote``,
    :216-247; a certificate it completes is processed at once, :244); a certificate goes to its
    round's ``CertificatesAggregator`` (``process_certificate``, :285-296).  Returns (errors per
    message, certificates assembled from votes, (parents, round) hand-offs to the proposer), i.e.
    what ``Core`` logs, broadcasts and sends on ``tx_proposer``.

    ``pipeline(batches)`` is the asynchronous form of the same loop: while batch k's verdicts are
    applied on the calling thread, batch k+1's state-independent checks (every digest and
    signature: ``check_messages``) already run on the GPU from a worker thread (ctypes releases the
    GIL during the library calls).  The state-dependent checks (TooOld against gc_round,
    UnexpectedVote against the current header) are evaluated when a batch is applied, against the
    state at that moment, so the results equal ``submit`` called batch after batch."""

    def __init__(self, committee: Committee, engine=None, gc_depth: int = 50):
        self.committee = committee
        self.engine = engine or _lib.default_engine()
        self.gc_depth = gc_depth
        self.gc_round = 0
        self.current_header = Header(bytes(32), 0)
        self.votes_aggregator = VotesAggregator()
        self.certificates_aggregators: Dict[int, CertificatesAggregator] = {}
        self.cert_base = 0   # global certificate index: the batch coefficients' stream position
        self.trace: Optional[list] = None   # pipeline event log (tests)

    def set_current_header(self, header: Header) -> None:
        """process_own_header (core.rs:117-120): a fresh votes aggregator for our new header."""
        self.current_header = header
        self.votes_aggregator = VotesAggregator()

    def _process_certificate(self, cert: Certificate, parents_out: list) -> None:
        agg = self.certificates_aggregators.setdefault(cert.round(), CertificatesAggregator())
        parents = agg.append(cert, self.committee)
        if parents is not None:
            parents_out.append((parents, cert.round()))

    def _check(self, messages: Sequence, zseed: Optional[bytes]):
        base = self.cert_base
        self.cert_base += sum(isinstance(m, Certificate) for m in messages)
        return check_messages(messages, self.committee, self.engine, zseed, base)

    def _apply(self, messages: Sequence, checked: List[Optional[DagError]]):
        errs: List[Optional[DagError]] = []
        assembled: List[Certificate] = []
        parents: List[Tuple[List[Certificate], int]] = []
        for m, e in zip(messages, checked):
            st = state_error(m, self.gc_round, self.current_header)
            err = st if st is not None else e
            if err is None and isinstance(m, Vote):
                try:
                    cert = self.votes_aggregator.append(m, self.committee, self.current_header)
                except DagError as ex:
                    err = ex
                else:
                    if cert is not None:
                        assembled.append(cert)
                        self._process_certificate(cert, parents)
            elif err is None and isinstance(m, Certificate):
                self._process_certificate(m, parents)
            errs.append(err)
        return errs, assembled, parents

    def submit(self, messages: Sequence, zseed: Optional[bytes] = None):
        return self._apply(messages, self._check(messages, zseed))

    def pipeline(self, batches: Iterable[Sequence], zseed: Optional[bytes] = None,
                 before_apply: Optional[Callable[[int, "CoreBatcher"], None]] = None):
        """Yield ``submit``'s result for each batch while the next batch is checked on the GPU.
        ``before_apply(k, self)`` runs on the calling thread just before batch k is applied (a
        hook for the state changes Core sees between messages: set_current_header, advance_gc)."""
        from concurrent.futures import ThreadPoolExecutor
        it = iter(batches)
        trace = self.trace

        def check(k, msgs):
            if trace is not None:
                trace.append(("check_start", k))
            r = self._check(msgs, zseed)
            if trace is not None:
                trace.append(("check_done", k))
            return r

        with ThreadPoolExecutor(max_workers=1) as ex:
            k = 0
            cur = next(it, None)
            fut = ex.submit(check, 0, cur) if cur is not None else None
            while cur is not None:
                nxt = next(it, None)
                checked = fut.result()
                fut = ex.submit(check, k + 1, nxt) if nxt is not None else None   # overlaps the apply below
                if trace is not None and nxt is not None:
                    trace.append(("submitted", k + 1))
                if before_apply is not None:
                    before_apply(k, self)
                res = self._apply(cur, checked)
                if trace is not None:
                    trace.append(("apply_done", k))
                yield res
                cur, k = nxt, k + 1

    def advance_gc(self, consensus_round: int) -> None:
        """The cleanup at the end of each Core::run iteration (core.rs:399-409)."""
        if consensus_round > self.gc_depth:
            self.gc_round = consensus_round - self.gc_depth
            self.certificates_aggregators = {r: a for r, a in self.certificates_aggregators.items()
                                             if r >= self.gc_round}
