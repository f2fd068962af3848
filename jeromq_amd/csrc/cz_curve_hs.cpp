// cz_curve_hs.cpp -- the CURVE handshake state machine (HELLO / WELCOME / INITIATE / READY), host
// side, with every public-key and secret-key operation on the GPU (cz_box / cz_box_open /
// cz_secretbox / cz_box_beforenm / cz_scalarmult, section 9 of the header).
//
// Mirrors, state for state and check for check:
//   CurveClientMechanism: constructor (ephemeral key pair, cnNonce = cnPeerNonce = 1) :55-78,
//     nextHandshakeCommand :80-103, processHandshakeCommand :105-124, status :227-239,
//     produceHello :246-279, processWelcome :281-316, produceInitiate :318-385,
//     processReady :387-419, processError :421-429
//   CurveServerMechanism: constructor :55-75, nextHandshakeCommand :77-106,
//     processHandshakeCommand :108-126, zapMsgAvailable :227-239, status :241-252,
//     processHello :254-299, produceWelcome :301-358, processInitiate :360-471,
//     produceReady :473-507, produceError :509-517
//   Mechanism: addProperty :101-116, parseMetadata :140-165, compare :182-185,
//     parseErrorMessage :218-241, handleErrorReason :243-263
//   Metadata.read (zmq/io/Metadata.java:365-417), Sockets.compatible (zmq/socket/Sockets.java:241-244),
//   Msgs.startsWith (zmq/io/Msgs.java:20-39).
// Events are the ZMQ_PROTOCOL_ERROR_* codes the reference passes to eventHandshakeFailedProtocol.
//
// Where the reference would throw (a READY or INITIATE larger than its fixed ByteBuffers, metadata
// over 256 bytes) this returns CZ_EPROTO / CZ_EMSGSIZE instead.  ZAP (RFC 27) is out of scope
// (SURVEY.md section 2): with zap enabled the server stops in EXPECT_ZAP_REPLY and the caller
// supplies the status code (cz_hs_zap_reply), which is what zapMsgAvailable consumes.
#include <sys/random.h>

#include <cstring>
#include <string>
#include <utility>
#include <vector>

#include "cz_internal.h"

using namespace czi;

namespace {

enum State {
    // client
    SEND_HELLO, EXPECT_WELCOME, SEND_INITIATE, EXPECT_READY, ERROR_RECEIVED,
    // server
    EXPECT_HELLO, SEND_WELCOME, EXPECT_INITIATE, EXPECT_ZAP_REPLY, SEND_READY, SEND_ERROR, ERROR_SENT,
    // both
    CONNECTED
};

// zmq/socket/Sockets.java: names by ZMQ_* type (the enum ordinal) and their compatible peers
struct SockType {
    const char *name;
    const char *peers[3];
};
const SockType SOCK_TYPES[] = {
    {"PAIR", {"PAIR"}},          {"PUB", {"SUB", "XSUB"}},       {"SUB", {"PUB", "XPUB"}},
    {"REQ", {"REP", "ROUTER"}},  {"REP", {"REQ", "DEALER"}},     {"DEALER", {"REP", "DEALER", "ROUTER"}},
    {"ROUTER", {"REQ", "DEALER", "ROUTER"}}, {"PULL", {"PUSH"}}, {"PUSH", {"PULL"}},
    {"XPUB", {"SUB", "XSUB"}},   {"XSUB", {"PUB", "XPUB"}},      {"STREAM", {}},
    {"SERVER", {"CLIENT"}},      {"CLIENT", {"SERVER"}},         {"RADIO", {"DISH"}},
    {"DISH", {"RADIO"}},         {"CHANNEL", {"CHANNEL"}},       {"PEER", {"PEER"}},
    {"RAW", {}},                 {"SCATTER", {"GATHER"}},        {"GATHER", {"SCATTER"}},
};
constexpr int NSOCK = (int)(sizeof(SOCK_TYPES) / sizeof(SOCK_TYPES[0]));
constexpr int ZMQ_REQ = 3, ZMQ_DEALER = 5, ZMQ_ROUTER = 6;

bool compatible(int self, const std::string &peer)
{
    if (self < 0 || self >= NSOCK)
        return false;
    for (const char *p : SOCK_TYPES[self].peers)
        if (p && peer == p)
            return true;
    return false;
}

// Msgs.startsWith(msg, data, true): the length byte, then bytes 1..len-1 against data[0..len-2]
// (the loop never reaches the last character: the reference's quirk, mirrored)
bool starts_with(const uint8_t *m, uint64_t size, const char *data)
{
    const uint64_t len = strlen(data);
    if (size < len + 1 || m[0] != len)
        return false;
    for (uint64_t i = 1; i < len; i++)
        if (m[i] != (uint8_t)data[i - 1])
            return false;
    return true;
}

uint64_t get_be64(const uint8_t *p)
{
    uint64_t v = 0;
    for (int i = 0; i < 8; i++)
        v = (v << 8) | p[i];
    return v;
}

void put_be64(uint8_t *p, uint64_t v)
{
    for (int i = 7; i >= 0; i--, v >>= 8)
        p[i] = (uint8_t)v;
}

// Mechanism.addProperty: name length byte, name, BE32 value length, value
void add_property(std::vector<uint8_t> &b, const char *name, const uint8_t *value, uint32_t vlen)
{
    const size_t n = strlen(name);
    b.push_back((uint8_t)n);
    b.insert(b.end(), name, name + n);
    for (int s = 24; s >= 0; s -= 8)
        b.push_back((uint8_t)(vlen >> s));
    if (vlen)
        b.insert(b.end(), value, value + vlen);
}

typedef std::vector<std::pair<std::string, std::vector<uint8_t>>> Props;

// Metadata.read + Mechanism.parseMetadata's listener: CZ_OK, CZ_EPROTO (trailing bytes that are not
// a whole property) or CZ_EINVAL (a Socket-Type the local type is not compatible with)
int parse_metadata(const uint8_t *buf, uint64_t len, int self_type, Props *out)
{
    uint64_t left = len, i = 0;
    while (left > 1) {
        const uint32_t nl = buf[i];
        if (nl == 0)
            break;
        i++;
        left--;
        if (left < nl)
            break;
        std::string name((const char *)buf + i, nl);
        i += nl;
        left -= nl;
        if (left < 4)
            break;
        const int32_t vl = (int32_t)(((uint32_t)buf[i] << 24) | ((uint32_t)buf[i + 1] << 16) |
                                     ((uint32_t)buf[i + 2] << 8) | buf[i + 3]);
        i += 4;
        left -= 4;
        if (vl < 0 || left < (uint64_t)vl)
            break;
        std::string value((const char *)buf + i, (size_t)vl);
        if (name == "Socket-Type" && !compatible(self_type, value))
            return CZ_EINVAL;
        if (out)
            out->push_back({name, std::vector<uint8_t>(buf + i, buf + i + vl)});
        i += (uint64_t)vl;
        left -= (uint64_t)vl;
    }
    return left > 0 ? CZ_EPROTO : CZ_OK;
}

// Wipe secret bytes with stores the compiler may not drop (a memset just before delete or a
// return is a dead store it is allowed to remove).
void secure_wipe(void *p, size_t n)
{
    explicit_bzero(p, n);
}

void secure_wipe(std::vector<uint8_t> &v)
{
    if (!v.empty())
        explicit_bzero(v.data(), v.size());
}

}  // namespace

struct cz_hs {
    bool server = false;
    State state = SEND_HELLO;
    int device = 0;
    int socket_type = 0;
    std::vector<uint8_t> identity;
    uint8_t pub[32] = {}, sec[32] = {}, server_key[32] = {};
    uint8_t cn_public[32] = {}, cn_secret[32] = {};
    uint8_t cn_peer_key[32] = {};  // client: S' (cnServer); server: C' (cnClient)
    uint8_t cn_cookie[96] = {};    // client: the WELCOME cookie
    uint8_t cookie_key[32] = {};   // server
    uint8_t cn_precom[32] = {};
    uint64_t cn_nonce = 1, cn_peer_nonce = 1;
    bool zap = false;
    std::string status_code;       // ZAP status ("200" ...); empty = none (produceError sends "")
    bool have_status = false;
    std::vector<uint8_t> client_key;  // server: the client's long-term key C from INITIATE
    Props peer;
    int event = 0;
    int auth_status = 0;          // client: status code of an ERROR from the server (handleErrorReason)
    // deterministic entropy (tests): random() draws come from here in order
    std::vector<uint8_t> entropy;
    size_t entropy_pos = 0;
    bool det = false;

    ~cz_hs()
    {
        secure_wipe(cn_secret, 32);
        secure_wipe(sec, 32);
        secure_wipe(cookie_key, 32);
        secure_wipe(cn_precom, 32);
        secure_wipe(entropy);
    }

    int random(uint8_t *out, size_t n)
    {
        if (det) {
            if (entropy_pos + n > entropy.size())
                return fail(CZ_EINVAL, "cz_hs: injected entropy exhausted");
            memcpy(out, entropy.data() + entropy_pos, n);
            entropy_pos += n;
            return CZ_OK;
        }
        size_t got = 0;
        while (got < n) {
            ssize_t r = getrandom(out + got, n - got, 0);
            if (r < 0)
                return fail(CZ_EINVAL, "cz_hs: getrandom failed");
            got += (size_t)r;
        }
        return CZ_OK;
    }

    int proto(int ev)
    {
        event = ev;
        return CZ_EPROTO;
    }

    // Box / open with the NaCl ZEROBYTES layouts (Curve.box / Curve.open, Curve.java:149-193)
    static int box(std::vector<uint8_t> &c, const std::vector<uint8_t> &m, const uint8_t n[24], const uint8_t pk[32],
                   const uint8_t sk[32])
    {
        c.assign(m.size(), 0);
        return cz_box(c.data(), m.data(), m.size(), n, pk, sk);
    }

    std::vector<uint8_t> metadata() const
    {
        std::vector<uint8_t> b;
        const char *tn = socket_type >= 0 && socket_type < NSOCK ? SOCK_TYPES[socket_type].name : "";
        add_property(b, "Socket-Type", (const uint8_t *)tn, (uint32_t)strlen(tn));
        if (socket_type == ZMQ_REQ || socket_type == ZMQ_DEALER || socket_type == ZMQ_ROUTER)
            add_property(b, "Identity", identity.data(), (uint32_t)identity.size());
        return b;
    }

    // ---- client ----
    int produce_hello(std::vector<uint8_t> &msg)
    {
        uint8_t nonce[24];
        memcpy(nonce, "CurveZMQHELLO---", 16);
        put_be64(nonce + 16, cn_nonce);
        std::vector<uint8_t> m(32 + 64, 0), c;
        if (box(c, m, nonce, server_key, cn_secret) != 0) {
            event = CZ_ZMTP_CRYPTOGRAPHIC;
            return -1;
        }
        msg.clear();
        const uint8_t head[] = {5, 'H', 'E', 'L', 'L', 'O', 1, 0};
        msg.insert(msg.end(), head, head + 8);
        msg.insert(msg.end(), 72, 0);
        msg.insert(msg.end(), cn_public, cn_public + 32);
        msg.insert(msg.end(), nonce + 16, nonce + 24);
        msg.insert(msg.end(), c.begin() + 16, c.begin() + 96);
        cn_nonce++;
        return CZ_OK;
    }

    int process_welcome(const uint8_t *m, uint64_t size)
    {
        if (size != 168)
            return proto(CZ_ZMTP_MALFORMED_COMMAND_READY);  // sic: the reference's event for a bad WELCOME
        std::vector<uint8_t> c(16 + 144, 0), p(c.size());
        memcpy(c.data() + 16, m + 24, 144);
        uint8_t nonce[24];
        memcpy(nonce, "WELCOME-", 8);
        memcpy(nonce + 8, m + 8, 16);
        if (cz_box_open(p.data(), c.data(), c.size(), nonce, server_key, cn_secret) != 0)
            return proto(CZ_ZMTP_CRYPTOGRAPHIC);
        memcpy(cn_peer_key, p.data() + 32, 32);
        memcpy(cn_cookie, p.data() + 64, 96);
        secure_wipe(p);
        if (cz_box_beforenm(cn_precom, cn_peer_key, cn_secret) != 0)
            return fail(CZ_EHIP, "cz_hs: beforenm failed");
        state = SEND_INITIATE;
        return CZ_OK;
    }

    int produce_initiate(std::vector<uint8_t> &msg)
    {
        uint8_t vnonce[24];
        memcpy(vnonce, "VOUCH---", 8);
        if (random(vnonce + 8, 16) != CZ_OK)
            return -1;
        std::vector<uint8_t> vm(32 + 64, 0), vc;
        memcpy(vm.data() + 32, cn_public, 32);
        memcpy(vm.data() + 64, server_key, 32);
        if (box(vc, vm, vnonce, cn_peer_key, sec) != 0) {
            event = CZ_ZMTP_CRYPTOGRAPHIC;
            return -1;
        }
        std::vector<uint8_t> im(32, 0);
        im.insert(im.end(), pub, pub + 32);
        im.insert(im.end(), vnonce + 8, vnonce + 24);
        im.insert(im.end(), vc.begin() + 16, vc.begin() + 96);
        const std::vector<uint8_t> meta = metadata();
        if (meta.size() > 256)  // "Assume here that metadata is limited to 256 bytes"
            return fail(CZ_EMSGSIZE, "cz_hs: INITIATE metadata of %zu bytes exceeds 256", meta.size());
        im.insert(im.end(), meta.begin(), meta.end());
        uint8_t nonce[24];
        memcpy(nonce, "CurveZMQINITIATE", 16);
        put_be64(nonce + 16, cn_nonce);
        std::vector<uint8_t> ic;
        if (box(ic, im, nonce, cn_peer_key, cn_secret) != 0) {
            event = CZ_ZMTP_CRYPTOGRAPHIC;
            return -1;
        }
        msg.clear();
        const char head[] = "\x08INITIATE";
        msg.insert(msg.end(), head, head + 9);
        msg.insert(msg.end(), cn_cookie, cn_cookie + 96);
        msg.insert(msg.end(), nonce + 16, nonce + 24);
        msg.insert(msg.end(), ic.begin() + 16, ic.end());
        cn_nonce++;
        return CZ_OK;
    }

    int process_ready(const uint8_t *m, uint64_t size)
    {
        if (size < 30)
            return proto(CZ_ZMTP_MALFORMED_COMMAND_READY);
        const uint64_t clen = 16 + size - 14;
        if (clen > 16 + 16 + 256)  // the reference's readyBox capacity (it would throw)
            return proto(CZ_ZMTP_MALFORMED_COMMAND_READY);
        std::vector<uint8_t> c(clen, 0), p(clen);
        memcpy(c.data() + 16, m + 14, size - 14);
        uint8_t nonce[24];
        memcpy(nonce, "CurveZMQREADY---", 16);
        memcpy(nonce + 16, m + 6, 8);
        cn_peer_nonce = get_be64(m + 6);
        if (cz_box_open_afternm(p.data(), c.data(), clen, nonce, cn_precom) != 0)
            return proto(CZ_ZMTP_CRYPTOGRAPHIC);
        peer.clear();
        const int rc = parse_metadata(p.data() + 32, clen - 32, socket_type, &peer);
        if (rc == CZ_OK)
            state = CONNECTED;
        return rc;
    }

    int process_error(const uint8_t *m, uint64_t size)
    {
        if (state != EXPECT_WELCOME && state != EXPECT_READY)
            return proto(CZ_ZMTP_UNEXPECTED_COMMAND);
        state = ERROR_RECEIVED;
        // Mechanism.parseErrorMessage
        if (size < 7 && size != 6)
            return proto(CZ_ZMTP_MALFORMED_COMMAND_ERROR);
        if (size >= 7) {
            const int8_t reason_len = (int8_t)m[6];  // a Java byte
            if (reason_len > (int64_t)size - 7)
                return proto(CZ_ZMTP_MALFORMED_COMMAND_ERROR);
            if (size == 10) {
                // handleErrorReason: "3xx".."5xx" with "00" -> handshake-failed-auth event
                const char a = (char)m[7], b = (char)m[8], d = (char)m[9];
                if (b == '0' && d == '0' && a >= '3' && a <= '5') {
                    auth_status = (a - '0') * 100;
                } else {
                    event = CZ_ZAP_MALFORMED_REPLY;
                    return CZ_EPROTO;
                }
            }
        }
        return CZ_OK;
    }

    // ---- server ----
    int process_hello(const uint8_t *m, uint64_t size)
    {
        if (!starts_with(m, size, "HELLO"))
            return proto(CZ_ZMTP_UNEXPECTED_COMMAND);
        if (size != 200)
            return proto(CZ_ZMTP_MALFORMED_COMMAND_HELLO);
        if (m[6] != 1 || m[7] != 0)
            return proto(CZ_ZMTP_MALFORMED_COMMAND_HELLO);
        memcpy(cn_peer_key, m + 80, 32);
        uint8_t nonce[24];
        memcpy(nonce, "CurveZMQHELLO---", 16);
        memcpy(nonce + 16, m + 112, 8);
        cn_peer_nonce = get_be64(m + 112);
        std::vector<uint8_t> c(16 + 80, 0), p(c.size());
        memcpy(c.data() + 16, m + 120, 80);
        if (cz_box_open(p.data(), c.data(), c.size(), nonce, cn_peer_key, sec) != 0) {
            event = CZ_ZMTP_CRYPTOGRAPHIC;  // the server answers with ERROR (status code null)
            state = SEND_ERROR;
            have_status = false;
            status_code.clear();
            return CZ_OK;
        }
        state = SEND_WELCOME;
        return CZ_OK;
    }

    int produce_welcome(std::vector<uint8_t> &msg)
    {
        uint8_t cnonce[24];
        memcpy(cnonce, "COOKIE--", 8);
        if (random(cnonce + 8, 16) != CZ_OK)
            return -1;
        std::vector<uint8_t> km(32 + 64, 0), kc(km.size(), 0);
        memcpy(km.data() + 32, cn_peer_key, 32);
        memcpy(km.data() + 64, cn_secret, 32);
        if (random(cookie_key, 32) != CZ_OK)
            return -1;
        if (cz_secretbox(kc.data(), km.data(), km.size(), cnonce, cookie_key) != 0)
            return fail(CZ_EHIP, "cz_hs: cookie secretbox failed");
        secure_wipe(km);  // held s'
        uint8_t wnonce[24];
        memcpy(wnonce, "WELCOME-", 8);
        if (random(wnonce + 8, 16) != CZ_OK)
            return -1;
        std::vector<uint8_t> wm(32, 0), wc;
        wm.insert(wm.end(), cn_public, cn_public + 32);
        wm.insert(wm.end(), cnonce + 8, cnonce + 24);
        wm.insert(wm.end(), kc.begin() + 16, kc.begin() + 96);
        if (box(wc, wm, wnonce, cn_peer_key, sec) != 0)
            return -1;
        msg.clear();
        const char head[] = "\x07WELCOME";
        msg.insert(msg.end(), head, head + 8);
        msg.insert(msg.end(), wnonce + 8, wnonce + 24);
        msg.insert(msg.end(), wc.begin() + 16, wc.begin() + 160);
        return CZ_OK;
    }

    int process_initiate(const uint8_t *m, uint64_t size)
    {
        if (!starts_with(m, size, "INITIATE"))
            return proto(CZ_ZMTP_UNEXPECTED_COMMAND);
        if (size < 257)
            return proto(CZ_ZMTP_MALFORMED_COMMAND_INITIATE);
        const uint64_t clen = size - 113 + 16;
        if (clen > 16 + 144 + 256)  // the reference's initiateBox capacity (it would throw)
            return proto(CZ_ZMTP_MALFORMED_COMMAND_INITIATE);
        // cookie = Box [C' + s'](t)
        std::vector<uint8_t> kc(16 + 80, 0), kp(kc.size());
        memcpy(kc.data() + 16, m + 25, 80);
        uint8_t cnonce[24];
        memcpy(cnonce, "COOKIE--", 8);
        memcpy(cnonce + 8, m + 9, 16);
        if (cz_secretbox_open(kp.data(), kc.data(), kc.size(), cnonce, cookie_key) != 0)
            return proto(CZ_ZMTP_CRYPTOGRAPHIC);
        const bool cookie_ok = memcmp(kp.data() + 32, cn_peer_key, 32) == 0 && memcmp(kp.data() + 64, cn_secret, 32) == 0;
        secure_wipe(kp);  // the cookie plaintext holds s'
        if (!cookie_ok)
            return proto(CZ_ZMTP_CRYPTOGRAPHIC);
        // Box [C + vouch + metadata](C'->S')
        std::vector<uint8_t> ic(clen, 0), ip(clen);
        memcpy(ic.data() + 16, m + 113, size - 113);
        uint8_t inonce[24];
        memcpy(inonce, "CurveZMQINITIATE", 16);
        memcpy(inonce + 16, m + 105, 8);
        cn_peer_nonce = get_be64(m + 105);
        if (cz_box_open(ip.data(), ic.data(), clen, inonce, cn_peer_key, cn_secret) != 0)
            return proto(CZ_ZMTP_CRYPTOGRAPHIC);
        client_key.assign(ip.begin() + 32, ip.begin() + 64);
        // vouch = Box [C',S](C->S'): must hold C'
        std::vector<uint8_t> vc(16 + 80, 0), vp(vc.size());
        memcpy(vc.data() + 16, ip.data() + 32 + 48, 80);
        uint8_t vnonce[24];
        memcpy(vnonce, "VOUCH---", 8);
        memcpy(vnonce + 8, ip.data() + 32 + 32, 16);
        if (cz_box_open(vp.data(), vc.data(), vc.size(), vnonce, client_key.data(), cn_secret) != 0)
            return proto(CZ_ZMTP_CRYPTOGRAPHIC);
        const bool vouch_ok = memcmp(vp.data() + 32, cn_peer_key, 32) == 0;
        secure_wipe(vp);
        if (!vouch_ok) {
            secure_wipe(ip);
            return proto(CZ_ZMTP_KEY_EXCHANGE);
        }
        if (cz_box_beforenm(cn_precom, cn_peer_key, cn_secret) != 0) {
            secure_wipe(ip);
            return fail(CZ_EHIP, "cz_hs: beforenm failed");
        }
        state = zap ? EXPECT_ZAP_REPLY : SEND_READY;
        peer.clear();
        const int mrc = parse_metadata(ip.data() + 32 + 128, clen - 32 - 128, socket_type, &peer);
        secure_wipe(ip);
        return mrc;
    }

    int produce_ready(std::vector<uint8_t> &msg)
    {
        std::vector<uint8_t> rm(32, 0);
        const std::vector<uint8_t> meta = metadata();
        if (meta.size() > 256)
            return fail(CZ_EMSGSIZE, "cz_hs: READY metadata of %zu bytes exceeds 256", meta.size());
        rm.insert(rm.end(), meta.begin(), meta.end());
        uint8_t nonce[24];
        memcpy(nonce, "CurveZMQREADY---", 16);
        put_be64(nonce + 16, cn_nonce);
        std::vector<uint8_t> rc(rm.size(), 0);
        if (cz_box_afternm(rc.data(), rm.data(), rm.size(), nonce, cn_precom) != 0)
            return fail(CZ_EHIP, "cz_hs: READY box failed");
        msg.clear();
        const char head[] = "\x05READY";
        msg.insert(msg.end(), head, head + 6);
        msg.insert(msg.end(), nonce + 16, nonce + 24);
        msg.insert(msg.end(), rc.begin() + 16, rc.end());
        cn_nonce++;
        return CZ_OK;
    }

    int produce_error(std::vector<uint8_t> &msg)
    {
        msg.clear();
        const char head[] = "\x05" "ERROR";
        msg.insert(msg.end(), head, head + 6);
        const std::string sc = have_status ? status_code : std::string();
        msg.push_back((uint8_t)sc.size());
        msg.insert(msg.end(), sc.begin(), sc.end());
        return CZ_OK;
    }

    // Mechanism.nextHandshakeCommand
    int next(std::vector<uint8_t> &msg)
    {
        int rc;
        switch (state) {
        case SEND_HELLO:
            rc = produce_hello(msg);
            if (rc == 0)
                state = EXPECT_WELCOME;
            return rc;
        case SEND_INITIATE:
            rc = produce_initiate(msg);
            if (rc == 0)
                state = EXPECT_READY;
            return rc;
        case SEND_WELCOME:
            rc = produce_welcome(msg);
            if (rc == 0)
                state = EXPECT_INITIATE;
            return rc;
        case SEND_READY:
            rc = produce_ready(msg);
            if (rc == 0)
                state = CONNECTED;
            return rc;
        case SEND_ERROR:
            rc = produce_error(msg);
            if (rc == 0)
                state = ERROR_SENT;
            return rc;
        default:
            return CZ_EAGAIN;
        }
    }

    // Mechanism.processHandshakeCommand
    int process(const uint8_t *m, uint64_t size)
    {
        if (!server) {
            // The reference client dispatches on the command name whatever its state
            // (CurveClientMechanism.java:108-129).  Deliberately stricter here, because this state
            // machine hands its session key straight to cz_engine / cz_mech: a READY before any
            // WELCOME would be opened under the all-zero cn_precom (a key anyone can compute) and
            // move the client to CONNECTED, and a WELCOME after CONNECTED would re-key the session.
            // So WELCOME is accepted only in EXPECT_WELCOME and READY only in EXPECT_READY.
            if (size >= 8 && starts_with(m, size, "WELCOME"))
                return state == EXPECT_WELCOME ? process_welcome(m, size) : proto(CZ_ZMTP_UNEXPECTED_COMMAND);
            if (size >= 6 && starts_with(m, size, "READY"))
                return state == EXPECT_READY ? process_ready(m, size) : proto(CZ_ZMTP_UNEXPECTED_COMMAND);
            if (size >= 6 && starts_with(m, size, "ERROR"))
                return process_error(m, size);
            return proto(CZ_ZMTP_UNEXPECTED_COMMAND);
        }
        switch (state) {
        case EXPECT_HELLO: return process_hello(m, size);
        case EXPECT_INITIATE: return process_initiate(m, size);
        default: return proto(CZ_ZMTP_UNSPECIFIED);
        }
    }

    int status() const
    {
        if (state == CONNECTED)
            return CZ_HS_READY;
        if (state == ERROR_RECEIVED || state == ERROR_SENT)
            return CZ_HS_ERROR;
        return CZ_HS_HANDSHAKING;
    }
};

extern "C" {

int cz_hs_create(cz_hs **out, int as_server, const uint8_t public_key[32], const uint8_t secret_key[32],
                 const uint8_t server_key[32], int socket_type, const uint8_t *identity, uint32_t identity_len,
                 const uint8_t *ephemeral_secret, const uint8_t *entropy, uint32_t entropy_len)
{
    if (!out)
        return fail(CZ_EINVAL, "cz_hs_create: null pointer");
    *out = nullptr;
    if (!secret_key || (!as_server && (!public_key || !server_key)) || (identity_len && !identity) ||
        (entropy_len && !entropy))
        return fail(CZ_EINVAL, "cz_hs_create: missing key");
    if (socket_type < 0 || socket_type >= NSOCK)
        return fail(CZ_EINVAL, "cz_hs_create: unknown socket type %d", socket_type);
    cz_hs *h = new cz_hs();
    h->server = as_server != 0;
    h->state = h->server ? EXPECT_HELLO : SEND_HELLO;
    h->socket_type = socket_type;
    if (identity_len)
        h->identity.assign(identity, identity + identity_len);
    memcpy(h->sec, secret_key, 32);
    if (public_key)
        memcpy(h->pub, public_key, 32);
    if (server_key)
        memcpy(h->server_key, server_key, 32);
    if (entropy) {
        h->det = true;
        h->entropy.assign(entropy, entropy + entropy_len);
    }
    // short-term key pair (Curve.keypair at construction); an injected secret is a test hook
    int rc;
    if (ephemeral_secret) {
        static const uint8_t nine[32] = {9};
        memcpy(h->cn_secret, ephemeral_secret, 32);
        rc = cz_scalarmult(h->cn_public, h->cn_secret, nine);
    } else {
        rc = cz_box_keypair(h->cn_public, h->cn_secret);
    }
    if (rc != 0) {
        delete h;
        return fail(CZ_EHIP, "cz_hs_create: ephemeral key pair needs the GPU (%s)", cz_last_error());
    }
    *out = h;
    return CZ_OK;
}

void cz_hs_destroy(cz_hs *h) { delete h; }

int cz_hs_next_command(cz_hs *h, uint8_t *out, uint32_t cap, uint32_t *len)
{
    if (!h || !len || (cap && !out))
        return fail(CZ_EINVAL, "cz_hs_next_command: null pointer");
    *len = 0;
    std::vector<uint8_t> msg;
    int rc = h->next(msg);
    if (rc == CZ_EAGAIN)
        return CZ_EAGAIN;
    if (rc != CZ_OK)
        return rc < 0 ? rc : CZ_EPROTO;
    if (msg.size() > cap)
        return fail(CZ_EMSGSIZE, "cz_hs_next_command: command of %zu bytes, buffer of %u", msg.size(), cap);
    memcpy(out, msg.data(), msg.size());
    *len = (uint32_t)msg.size();
    return CZ_OK;
}

int cz_hs_process_command(cz_hs *h, const uint8_t *cmd, uint64_t size)
{
    if (!h || (size && !cmd))
        return fail(CZ_EINVAL, "cz_hs_process_command: null pointer");
    static const uint8_t empty[1] = {0};
    return h->process(size ? cmd : empty, size);
}

int cz_hs_status(const cz_hs *h) { return h ? h->status() : CZ_EINVAL; }

int cz_hs_event(const cz_hs *h) { return h ? h->event : 0; }

int cz_hs_error_status(const cz_hs *h) { return h ? h->auth_status : 0; }

int cz_hs_set_zap(cz_hs *h, int on)
{
    if (!h || !h->server)
        return fail(CZ_EINVAL, "cz_hs_set_zap: not a server handshake");
    h->zap = on != 0;
    return CZ_OK;
}

int cz_hs_zap_reply(cz_hs *h, const char *status_code)
{
    if (!h || !status_code)
        return fail(CZ_EINVAL, "cz_hs_zap_reply: null pointer");
    if (h->state != EXPECT_ZAP_REPLY)
        return fail(CZ_EINVAL, "cz_hs_zap_reply: no ZAP reply expected (EFSM)");
    if (strlen(status_code) != 3) {
        h->event = CZ_ZAP_INVALID_STATUS_CODE;
        return CZ_EPROTO;
    }
    h->status_code = status_code;
    h->have_status = true;
    h->state = h->status_code == "200" ? SEND_READY : SEND_ERROR;
    return CZ_OK;
}

int cz_hs_client_key(const cz_hs *h, uint8_t key[32])
{
    if (!h || !key || h->client_key.size() != 32)
        return fail(CZ_EINVAL, "cz_hs_client_key: no INITIATE processed");
    memcpy(key, h->client_key.data(), 32);
    return CZ_OK;
}

int cz_hs_session(const cz_hs *h, uint8_t precom[32], uint64_t *cn_nonce, uint64_t *cn_peer_nonce)
{
    if (!h || !precom || !cn_nonce || !cn_peer_nonce)
        return fail(CZ_EINVAL, "cz_hs_session: null pointer");
    if (h->state != CONNECTED)
        return fail(CZ_EINVAL, "cz_hs_session: handshake not complete");
    memcpy(precom, h->cn_precom, 32);
    *cn_nonce = h->cn_nonce;
    *cn_peer_nonce = h->cn_peer_nonce;
    return CZ_OK;
}

int cz_hs_peer_property(const cz_hs *h, const char *name, const uint8_t **value, uint32_t *len)
{
    if (!h || !name || !value || !len)
        return fail(CZ_EINVAL, "cz_hs_peer_property: null pointer");
    for (const auto &p : h->peer)
        if (p.first == name) {
            *value = p.second.data();
            *len = (uint32_t)p.second.size();
            return CZ_OK;
        }
    return fail(CZ_EINVAL, "cz_hs_peer_property: no property %s", name);
}

cz_mech *cz_hs_mechanism(const cz_hs *h, int device)
{
    uint8_t k[32];
    uint64_t n, pn;
    if (cz_hs_session(h, k, &n, &pn) != CZ_OK)
        return nullptr;
    cz_mech *m = cz_mech_create(h->server ? 1 : 0, k, n, pn, device);
    secure_wipe(k, 32);
    return m;
}

int cz_engine_add_session(cz_engine *e, const cz_hs *h)
{
    uint8_t k[32];
    uint64_t n, pn;
    int rc = cz_hs_session(h, k, &n, &pn);
    if (rc != CZ_OK)
        return rc;
    rc = cz_engine_add_conn(e, h->server ? 1 : 0, k, n, pn);
    secure_wipe(k, 32);
    return rc;
}

int cz_zmtp_metadata_check(const uint8_t *buf, uint64_t len, int socket_type)
{
    if (len && !buf)
        return fail(CZ_EINVAL, "cz_zmtp_metadata_check: null pointer");
    return parse_metadata(buf, len, socket_type, nullptr);
}

uint32_t cz_zmtp_metadata(int socket_type, const uint8_t *identity, uint32_t identity_len, uint8_t *out, uint32_t cap)
{
    cz_hs h;
    h.socket_type = socket_type;
    if (identity_len && identity)
        h.identity.assign(identity, identity + identity_len);
    const std::vector<uint8_t> b = h.metadata();
    if (out && b.size() <= cap)
        memcpy(out, b.data(), b.size());
    return (uint32_t)b.size();
}

}  // extern "C"
