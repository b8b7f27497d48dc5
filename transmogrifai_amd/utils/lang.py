"""Language identification and language-aware analysis (replaces Optimaize ``LanguageDetector`` and the
per-language Lucene analyzers of ``LuceneTextAnalyzer.scala:87-236``; SURVEY.md L0 text interfaces).

* :func:`detect_languages` -- ``{ISO 639-1 code: confidence}``. Text in a non-Latin script is identified
  by its script (Cyrillic with Ukrainian letters -> uk, else ru; Greek, Arabic (Persian letters -> fa),
  Hebrew, Devanagari, Thai, Hangul, kana -> ja, Han only -> zh); Latin-script text by the share of
  each language's most frequent function words among its tokens (a stop-word profile in place of
  Optimaize's n-gram profiles, which are not available offline).
* :func:`analyze` -- the reference's per-language analysis: the language's stop words, elision stripping for
  French / Italian / Catalan (``l'amour`` -> ``amour``, Lucene ElisionFilter), English possessive removal
  and Porter stemming (``utils/stemmer.py``, Lucene EnglishAnalyzer), on top of the StandardAnalyzer word
  rules of :func:`utils.text.analyze`; the languages of ``utils/stemmers.py`` STEMMERS stem after their stop
  filter. Turkish (TurkishAnalyzer's Snowball stemmer) is not reproduced: its tokens are stop-filtered only.
"""
from __future__ import annotations

import unicodedata
from typing import Dict, FrozenSet, List, Optional

from . import text as TU

UNKNOWN = "Unknown"

_PROFILE = {
    "en": "the of and to in is that it was for on are with as his they be at one have this from by not but "
          "what all were we when your can said there use an each which she do how their if will",
    "fr": "le la les de des et un une est que qui dans pour pas sur au avec il elle nous vous ce cette sont "
          "du en aux ne se ses mais ou leur plus par je tu",
    "de": "der die das und ist nicht ein eine zu den mit von sie es ich auf auch dem des sich im für wie "
          "aber bei oder wir werden nach noch hat sind",
    "es": "el la los las de y que en un una es por con para no se su al lo como del más pero sus le ya "
          "o este fue ha muy sin sobre también",
    "it": "il lo la gli le di e che un una non per con sono nel della sul anche come del dei ma si è ha "
          "questo alla più era delle degli",
    "pt": "o a os as de e que em um uma não para com por se na no mais como do da dos das ao foi são "
          "ele ela mas tem seu sua",
    "nl": "de het een en van is dat niet te op zijn met voor er aan ook als die maar om ik je bij naar "
          "wordt heeft deze hij",
    "sv": "och att det som en på är av för med till den inte har de ett om jag var sig men så kan vi "
          "hade eller från",
    "da": "og at det som en på er af for med til den ikke har de et om jeg var sig men så kan vi havde "
          "eller fra",
    "no": "og i det som en på er av for med til den ikke har de et om jeg var seg men så kan vi hadde "
          "eller fra",
    "pl": "i w nie na się z że do jest to jak o po ale co tak czy od już przez być jego",
    "ca": "el la els les de i que en un una és per amb no es del al com més però dels",
    "fi": "ja on ei se että oli hän olla mutta kun ovat tai jos niin myös kuin",
    "tr": "ve bir bu da de için ile çok ama gibi daha olarak olan en ne var",
    "ro": "și în de la cu nu o un care este pe din să se ca mai",
    "cs": "a se na je že to v z do o s k ve jsou ale jak pro po by jako jsem už jeho které který není také",
    "id": "yang dan di ini itu dengan untuk tidak dari dalam akan pada juga ke karena tersebut bisa ada mereka adalah",
    "lv": "un ir ar uz no par kas ka bet lai arī vai pie pēc tas to viņš bija tā nav",
}
PROFILES: Dict[str, FrozenSet[str]] = {k: frozenset(v.split()) for k, v in _PROFILE.items()}

# stop words of the per-language analyzers (English: Lucene's english_stop list of utils/text.py)
STOPWORDS: Dict[str, FrozenSet[str]] = dict(PROFILES)
STOPWORDS["en"] = TU.ENGLISH_STOPWORDS
# FrenchAnalyzer's stop set (the Snowball French list)
STOPWORDS["fr"] = PROFILES["fr"] | frozenset("""
au aux avec ce ces dans de des du elle en et eux il je la le leur lui ma mais me même mes moi mon ne nos notre nous
on ou par pas pour qu que qui sa se ses son sur ta te tes toi ton tu un une vos votre vous c d j l à m n s t y été
étée étées étés étant étante étants étantes suis es est sommes êtes sont serai seras sera serons serez seront serais
serait serions seriez seraient étais était étions étiez étaient fus fut fûmes fûtes furent sois soit soyons soyez
soient fusse fusses fût fussions fussiez fussent ayant ayante ayantes ayants eu eue eues eus ai as avons avez ont
aurai auras aura aurons aurez auront aurais aurait aurions auriez auraient avais avait avions aviez avaient eut eûmes
eûtes eurent aie aies ait ayons ayez aient eusse eusses eût eussions eussiez eussent""".split())

# Snowball stop lists of the Russian and Dutch analyzers
STOPWORDS["ru"] = frozenset("""
и в во не что он на я с со как а то все она так его но да ты к у же вы за бы по только ее мне было вот от меня еще нет
о из ему теперь когда даже ну вдруг ли если уже или ни быть был него до вас нибудь опять уж вам ведь там потом себя
ничего ей может они тут где есть надо ней для мы тебя их чем была сам чтоб без будто чего раз тоже себе под будет ж
тогда кто этот того потому этого какой совсем ним здесь этом один почти мой тем чтобы нее сейчас были куда зачем всех
никогда можно при наконец два об другой хоть после над больше тот через эти нас про всего них какая много разве три
эту моя впрочем хорошо свою этой перед иногда лучше чуть том нельзя такой им более всегда конечно всю между""".split())
STOPWORDS["nl"] = PROFILES["nl"] | frozenset("""
de en van ik te dat die in een hij het niet zijn is was op aan met als voor had er maar om hem dan zou of wat mijn men
dit zo door over ze zich bij ook tot je mij uit der daar haar naar heb hoe heeft hebben deze u want nog zal me zij nu
ge geen omdat iets worden toch al waren veel meer doen toen moet ben zonder kan hun dus alles onder ja eens hier wie
werd altijd doch wordt wezen kunnen ons zelf tegen na reeds wil kon niets uw iemand geweest andere""".split())

# Snowball stop lists of the Finnish, Hungarian and Romanian analyzers (Lucene's RomanianAnalyzer list for ro)
STOPWORDS["fi"] = PROFILES["fi"] | frozenset("""
olla olen olet on olemme olette ovat ole oli olisi olisit olisin olisimme olisitte olisivat olit olin olimme olitte
olivat ollut olleet en et ei emme ette eivät minä minun minut minua minussa minusta minuun minulla minulta minulle sinä
sinun sinut sinua sinussa sinusta sinuun sinulla sinulta sinulle hän hänen hänet häntä hänessä hänestä häneen hänellä
häneltä hänelle me meidän meidät meitä meissä meistä meihin meillä meiltä meille te teidän teidät teitä teissä teistä
teihin teillä teiltä teille he heidän heidät heitä heissä heistä heihin heillä heiltä heille tämä tämän tätä tässä
tästä tähän tällä tältä tälle tänä täksi tuo tuon tuota tuossa tuosta tuohon tuolla tuolta tuolle tuona tuoksi se sen
sitä siinä siitä siihen sillä siltä sille sinä siksi nämä näiden näitä näissä näistä näihin näillä näiltä näille näinä
näiksi nuo noiden noita noissa noista noihin noilla noilta noille noina noiksi ne niiden niitä niissä niistä niihin
niillä niiltä niille niinä niiksi kuka kenen kenet ketä kenessä kenestä keneen kenellä keneltä kenelle kenenä keneksi
ketkä keiden keitä keissä keistä keihin keillä keiltä keille keinä keiksi mikä minkä mitä missä mistä mihin millä
miltä mille miksi mitkä joka jonka jota jossa josta johon jolla jolta jolle jona joksi jotka joiden joita joissa
joista joihin joilla joilta joille joina joiksi että ja jos koska kuin mutta niin sekä tai vaan vai vaikka kanssa
mukaan noin poikki yli kun nyt itse""".split())
STOPWORDS["hu"] = frozenset("""
a ahogy ahol aki akik akkor alatt által általában amely amelyek amelyekben amelyeket amelyet amelynek ami amit amolyan
amíg amikor át abban ahhoz annak arra arról az azok azon azt azzal azért aztán azután azonban bár be belül benne cikk
cikkek cikkeket csak de e eddig egész egy egyes egyetlen egyéb egyik egyre ekkor el elég ellen elő először előtt első
én éppen ebben ehhez emilyen ennek erre ez ezt ezek ezen ezzel ezért és fel felé hanem hiszen hogy hogyan igen így
illetve ill ilyen ilyenkor ismét itt jó jól jobban kell kellett keresztül keressünk ki kívül között közül legalább
lehet lehetett legyen lenne lenni lesz lett maga magát majd már más másik meg még mellett mert mely melyek mi mit míg
miért milyen mikor minden mindent mindenki mindig mint mintha mivel most nagy nagyobb nagyon ne néha nekem neki nem
néhány nélkül nincs olyan ott össze ő ők őket pedig persze rá s saját sem semmi sok sokat sokkal számára szemben
szerint szinte talán tehát teljes tovább továbbá több úgy ugyanis új újabb újra után utána utolsó vagy vagyis valaki
valami valamint való vagyok van vannak volt voltam voltak voltunk vissza vele viszont volna""".split())
STOPWORDS["ro"] = PROFILES["ro"] | frozenset("""
a abia acea aceasta această aceea acei aceia acel acela acele acelea acest acesta aceste acestea acestei acestia
acestui aceşti aceştia acolo acum ai aia aibă aici al ale alea alt alta altceva altcineva alte altfel alti altii altul
am anume apoi ar are as asa asta astazi astfel asupra atare atat atata atatea atatia ati atit atita atitea atitia
atunci au avea avem avut azi aş aşadar aţi ba bine bucur bună ca cand care careia carora caruia cat catre ce cea ceea
cei ceilalti cel cele celor ceva chiar ci cind cine cineva cit cita cite citeva citi citiva cu cui cum cumva da daca
dar dat dată de deasupra deci decit deja desi despre din dintr dintre doar doi doilea două drept dupa după ea ei el ele
era este eu exact eşti face fara fata fel fi fie fiecare fii fim fiu fiţi foarte fost fără geaba ia iar ii il imi in
inainte inapoi inca incit insa intr intre isi iti la le li lor lui ma mai mea mei mele mereu meu mi mie mine mod mult
multa multe multi mâine mîine ne ni nici nimeni nimic niste nişte noastre noastră noi nostri nostru nou noua nouă
noştri nu numai or ori oricare orice oricine oricum oricând oricît oriunde pai parca patra patru pe pentru peste pic
pina poate pot prea prima primul prin printr putini puţin puţina puţină până pînă sa sai sale sau se si sint sintem
spate spre sub sunt suntem sunteţi sus să săi său ta tale te ti tine toata toate toată tocmai tot toti totul totusi
totuşi toţi trei treia treilea tu tuturor tăi tău ul ului un una unde undeva unei uneia unele uneori unii unor unora
unu unui unuia unul va vi voastre voastră voi vom vor vostru vouă voştri vreo vreun vă zi zice îi îl îmi în îţi ăla
ălea ăsta ăstea ăştia şi ţi ţie""".split())

# ArabicAnalyzer's stop set (matched before normalisation, as its StopFilter runs first)
STOPWORDS["ar"] = frozenset("""
من ومن منها منه في وفي فيها فيه و ف ثم او أو ب بها به ا أ اى اي أي أى لا ولا الا ألا إلا لكن ما وما كما فما عن مع
اذا إذا ان أن إن انها أنها إنها انه أنه إنه بان بأن فان فأن وان وأن وإن التى التي الذى الذي الذين الى الي إلى إلي
على عليها عليه اما أما إما ايضا أيضا كل وكل لم ولم لن ولن هى هي هو وهى وهي وهو فهى فهي فهو انت أنت لك لها له هذه
هذا تلك ذلك هناك كانت كان يكون تكون وكانت وكان غير بعض قد نحو بين بينما منذ ضمن حيث الان الآن خلال بعد قبل حتى
عند عندما لدى جميع""".split())

# HindiAnalyzer's stop set (common function words of the Lucene list; matched before normalisation)
STOPWORDS["hi"] = frozenset("""
अंदर अत अदि अप अपना अपनि अपनी अपने अभि अभी आदि आप इंहिं इंहें इंहों इतयादि इत्यादि इन इनका इन्हीं इन्हें इन्हों इस इसका इसकि
इसकी इसके इसमें इसि इसी इसे उंहिं उंहें उंहों उन उनका उनकि उनकी उनके उनको उन्हीं उन्हें उन्हों उस उसके उसि उसी उसे एक एवं एस
एसे ऐसे ओर और कइ कई कर करता करते करना करने करें कहते कहा का काफि काफ़ी कि किंहें किंहों कितना किन्हें किन्हों किया किर किस
किसि किसी किसे की कुछ कुल के को कोइ कोई कोन कोनसा कौन कौनसा गया घर जब जहाँ जहां जा जिंहें जिंहों जितना जिधर जिन जिन्हें
जिन्हों जिस जिसे जीधर जेसा जेसे जैसा जैसे जो तक तब तरह तिंहें तिंहों तिन तिन्हें तिन्हों तिस तिसे तो था थि थी थे दबारा दवारा
दिया दुसरा दुसरे दूसरे दो द्वारा न नहिं नहीं ना निचे निहायत नीचे ने पर पहले पुरा पूरा पे फिर बनि बनी बहि बही बहुत बाद बाला
बिलकुल भि भितर भी भीतर मगर मानो मे में यदि यह यहाँ यहां यहि यही या यिह ये रखें रवासा रहा रहे ऱ्वासा लिए लिये लेकिन व वगेरह वरग
वर्ग वह वहाँ वहां वहिं वहीं वाले वुह वे वग़ैरह संग सकता सकते सबसे सभि सभी साथ साबुत साभ सारा से सो हि ही हुअ हुआ हुइ हुई
हुए हे हें है हैं हो होता होति होती होते होना होने""".split())

# BulgarianAnalyzer's stop set (Savoy's Bulgarian list, as shipped with Lucene)
STOPWORDS["bg"] = frozenset("""
а аз ако ала бе без беше би бил била били било близо бъдат бъде бяха в вас ваш ваша вероятно вече взема ви вие винаги
все всеки всички всичко всяка във въпреки върху г ги главно го д да дали до докато докога дори досега доста е едва
един ето за зад заедно заради засега затова защо защото и из или им има имат иска й каза как каква какво както какъв
като кога когато което които кой който колко която къде където към ли м ме между мен ми мнозина мога могат може моля
момента му н на над назад най направи напред например нас не него нея ни ние никой нито но някои някой няма обаче
около освен особено от отгоре отново още пак по повече повечето под поне поради после почти прави пред преди през
при пък първо с са само се сега си скоро след сме според сред срещу сте съм със също т тази така такива такъв там
твой те тези ти то това тогава този той толкова точно трябва тук тъй тя тях у харесва ч че често чрез ще щом я""".split())

# CzechAnalyzer's stop set
STOPWORDS["cs"] = PROFILES["cs"] | frozenset("""
a s k o i u v z dnes cz tímto budeš budem byli jseš můj svým ta tomto tohle tuto tyto jej zda proč máte tato kam
tohoto kdo kteří mi nám tom tomuto mít nic proto kterou byla toho protože asi ho naši napište re což tím takže svých
její svými jste aj tu tedy teto bylo kde ke pravé ji nad nejsou či pod téma mezi přes ty pak vám ani když však neg
jsem tento článku články aby jsme před pta jejich byl ještě až bez také pouze první vaše která nás nový tipy pokud
může strana jeho své jiné zprávy nové není vás jen podle zde už být více bude již než který by které co nebo ten
tak má při od po jsou jak další ale si se ve to jako za zpět ze do pro je na atd atp jakmile přičemž já on ona ono
oni ony my vy jí mě mne jemu tomu těm těmu němu němuž jehož jíž jelikož jež jakož načež""".split())

# PersianAnalyzer's stop set (normalised forms: its StopFilter runs after the normalisation filters)
STOPWORDS["tr"] = PROFILES["tr"] | frozenset("""
acaba altmış altı ama ancak arada aslında ayrıca bana bazı belki ben benden beni benim beri beş bile bin bir birçok
biri birkaç birkez birşey birşeyi biz bize bizden bizi bizim böyle böylece bu buna bunda bundan bunlar bunları
bunların bunu bunun burada çok çünkü da daha dahi de defa değil diğer diye doksan dokuz dolayı dolayısıyla dört
edecek eden ederek edilecek ediliyor edilmesi ediyor eğer elli en etmesi etti ettiği ettiğini gibi göre halen hangi
hatta hem henüz hep hepsi her herhangi herkesin hiç hiçbir için iki ile ilgili ise işte itibaren itibariyle kadar
karşın katrilyon kendi kendilerine kendini kendisi kendisine kendisini kez ki kim kimden kime kimi kimse kırk milyar
milyon mu mü mı nasıl ne neden nedenle nerde nerede nereye niye niçin o olan olarak oldu olduğu olduğunu olduklarını
olmadı olmadığı olmak olması olmayan olmaz olsa olsun olup olur olursa oluyor on ona ondan onlar onlardan onları
onların onu onun otuz oysa öyle pek rağmen sadece sanki sekiz seksen sen senden seni senin siz sizden sizi sizin şey
şeyden şeyi şeyler şöyle şu şuna şunda şundan şunları şunu tarafından trilyon tüm üç üzere var vardı ve veya ya
yani yapacak yapılan yapılması yapıyor yapmak yaptı yaptığı yaptığını yaptıkları yedi yerine yetmiş yine yirmi
yoksa yüz zaten""".split())
# IndonesianAnalyzer's stop set (F. Tala's list; its common entries)
STOPWORDS["id"] = PROFILES["id"] | frozenset("""
ada adalah adanya adapun agak agaknya agar akan akankah akhirnya aku akulah amat amatlah anda andalah antar antara
antaranya apa apaan apabila apakah apalagi apatah atau ataukah ataupun bagai bagaikan bagaimana bagaimanakah
bagaimanapun bagi bahkan bahwa bahwasanya banyak beberapa begini beginian beginikah beginilah begitu begitukah
begitulah begitupun belum belumlah berapa berapakah berapalah berapapun bermacam bersama betulkah biasa biasanya
bila bilakah bisa bisakah boleh bolehkah bolehlah buat bukan bukankah bukanlah bukannya cuma dahulu dalam dan dapat
dari daripada dekat demi demikian demikianlah dengan depan di dia dialah diantara diantaranya dikarenakan dini diri
dirinya disini disinilah dong dulu enggak enggaknya entah entahlah hal hampir hanya hanyalah harus haruslah
harusnya hendak hendaklah hendaknya hingga ia ialah ibarat ingin inginkah inginkan ini inikah inilah itu itukah
itulah jangan jangankan janganlah jika jikalau juga justru kala kalau kalaulah kalaupun kalian kami kamilah kamu
kamulah kan kapan kapankah kapanpun karena karenanya ke kecil kemudian kenapa kepada kepadanya ketika khususnya kini
kinilah kiranya kita kitalah kok lagi lagian lah lain lainnya lalu lama lamanya lebih macam maka makanya makin
malah malahan mampu mampukah mana manakala manalagi masih masihkah masing mau maupun melainkan melalui memang
mengapa mereka merekalah merupakan meski meskipun mungkin mungkinkah nah namun nanti nantinya nyaris oleh olehnya
pada padahal padanya paling pantas para pasti pastilah per percuma pernah pula pun rupanya saat saatnya saja
sajalah saling sama sambil sampai sana sangat sangatlah saya sayalah se sebab sebabnya sebagai sebagaimana
sebagainya sebaliknya sebanyak sebegini sebegitu sebelum sebelumnya sebenarnya seberapa sebetulnya sebisanya
sebuah sedang sedangkan sedemikian sedikit sedikitnya segala segalanya segera seharusnya sehingga sejak sejenak
sekali sekalian sekaligus sekalipun sekarang seketika sekiranya sekitar sekitarnya sela selagi selain selaku
selalu selama selamanya seluruh seluruhnya semacam semakin semasih semaunya sementara sempat semua semuanya semula
sendiri sendirinya seolah seorang sepanjang sepantasnya seperti sepertinya sering seringnya serta serupa sesaat
sesama sesegera sesuatu sesuatunya sesudah sesudahnya setelah seterusnya setiap setidaknya sewaktu siapa siapakah
siapapun sini sinilah suatu sudah sudahkah sudahlah supaya tadi tadinya tak tanpa tapi telah tentang tentu
tentulah tentunya terdiri terhadap terhadapnya terlalu terlebih tersebut tersebutlah tertentu tetapi tiap tidak
tidakkah tidaklah toh waduh wah wahai walau walaupun wong yaitu yakni yang""".split())
STOPWORDS["lv"] = PROFILES["lv"] | frozenset("""
aiz ap ar apakš ārpus augšpus bez caur dēļ gar iekš iz kopš labad lejpus līdz no otrpus pa par pār pēc pie pirms
pret priekš starp šaipus uz viņpus virs virspus zem apakšpus un bet jo ja ka lai tomēr tikko turpretī arī kaut gan
tādēļ tā ne tikvien vien kā ir te vai kamēr diezin droši diemžēl nebūt ik it taču nu pat tiklab iekšpus nedz tik
nevis turpretim jeb iekam iekām iekāms kolīdz līdzko tiklīdz jebšu tālab tāpēc nekā itin jā jau jel nē nezin tad
tikai vis tak iekams būt biju biji bija bijām bijāt esmu esi esam esat būšu būsi būs būsim būsiet tikt tiku tiki
tika tikām tikāt tieku tiec tiek tiekam tiekat tikšu tiks tiksim tiksiet tapt tapi tapāt topat tapšu tapsi taps
tapsim tapsiet kļūt kļuvu kļuvi kļuva kļuvām kļuvāt kļūstu kļūsti kļūst kļūstam kļūstat kļūšu kļūsi kļūs kļūsim
kļūsiet varēt varēju varējām varēšu varēsim var varēji varējāt varēsi varēsiet varat varēja varēs""".split())
STOPWORDS["fa"] = frozenset("""
انان نداشته سراسر خياه ايشان وي تاكنون بيشتري دوم پس ناشي وگو يا داشتند سپس هنگام هرگز پنج نشان امسال ديگر گروهي
شدند چطور ده و دو نخستين ولي چرا چه وسط ه كدام قابل يك رفت هفت همچنين در هزار بله بلي شايد اما شناسي گرفته دهد
داشته دانست داشتن خواهيم ميليارد وقتي امد خواهد جز اورده شده بلكه خدمات شدن برخي نبود بسياري جلوگيري حق كردند
نوعي بعري نكرده نظير نبايد بوده بودن داد اورد هست جايي شود دنبال داده بايد سابق هيچ همان انجا كمتر كجاست گردد كسي
تر مردم تان دادن بودند سري جدا ندارند مگر يكديگر دارد دهند بنابراين هنگامي سمت جا انچه خود دادند زياد دارند اثر
بدون بهترين بيشتر البته به براساس بيرون كرد بعضي گرفت توي اي ميليون او جريان تول بر مانند برابر باشيم مدتي گويند
اكنون تا تنها جديد چند بي نشده كردن كردم گويد كرده كنيم نمي نزد روي قصد فقط بالاي ديگران اين ديروز توسط سوم ايم
دانند سوي استفاده شما كنار داريم ساخته طور امده رفته نخست بيست نزديك طي كنيد از انها تمامي داشت يكي طريق اش چيست
روب نمايد گفت چندين چيزي تواند ام ايا با ان ايد ترين اينكه ديگري راه هايي بروز همچنان پاعين كس حدود مختلف مقابل
چيز گيرد ندارد ضد همچون سازي شان مورد باره مرسي خويش برخوردار چون خارج شش هنوز تحت ضمن هستيم گفته فكر بسيار پيش
براي روزهاي انكه نخواهد بالا كل كي چنين كه گيري نيست است كجا كند نيز يابد بندي حتي توانند عقب خواست كنند بين
تمام همه ما باشند مثل شد اري باشد اره طبق بعد اگر صورت غير جاي بيش ريزي اند زيرا چگونه بار لطفا مي درباره من
ديده همين گذاري برداري علت گذاشته هم فوق نه ها شوند اباد همواره هر اول خواهند چهار نام امروز مان هاي قبل كنم سعي
تازه را هستند زير جلوي عنوان بود""".split())

from .stemmers_more import STOPWORDS_MORE as _SW_MORE  # noqa: E402

STOPWORDS.update(_SW_MORE)
# IrishAnalyzer: its hyphenation prefixes (h-, n-, t-, split off by the tokenizer) are stopped with the stop words
STOPWORDS["ga"] = STOPWORDS["ga"] | frozenset(("h", "n", "t"))

_ELISIONS = {"fr": ("l", "m", "t", "qu", "n", "s", "j", "d", "c", "jusqu", "quoiqu", "lorsqu", "puisqu"),
             "it": ("c", "l", "all", "dall", "dell", "nell", "sull", "coll", "pell", "gl", "agl", "dagl",
                    "degl", "negl", "sugl", "un", "m", "t", "s", "v", "d"),
             "ca": ("d", "l", "m", "n", "s", "t"), "ga": ("d", "m", "b")}


def _script_counts(text: str) -> Dict[str, int]:
    c: Dict[str, int] = {}
    for ch in text:
        o = ord(ch)
        if o < 0x80:
            if ch.isalpha():
                c["Latin"] = c.get("Latin", 0) + 1
            continue
        if not ch.isalpha():
            continue
        if 0x3040 <= o <= 0x30FF:
            s = "Kana"
        elif 0xAC00 <= o <= 0xD7AF or 0x1100 <= o <= 0x11FF:
            s = "Hangul"
        elif 0x4E00 <= o <= 0x9FFF or 0x3400 <= o <= 0x4DBF:
            s = "Han"
        else:
            try:
                s = unicodedata.name(ch).split(" ")[0]
            except ValueError:
                continue
        c[s] = c.get(s, 0) + 1
    return c


_ODDS = 4.0

_SCRIPT_LANG = {"GREEK": "el", "HEBREW": "he", "DEVANAGARI": "hi", "THAI": "th", "Hangul": "ko", "BENGALI": "bn",
                "ARMENIAN": "hy", "GEORGIAN": "ka", "TAMIL": "ta"}


def detect_languages(text: Optional[str]) -> Dict[str, float]:
    if not text:
        return {}
    sc = _script_counts(text)
    letters = sum(sc.values())
    if letters == 0:
        return {}
    latin = sc.get("LATIN", 0) + sc.get("Latin", 0)
    out: Dict[str, float] = {}
    if sc.get("Kana", 0):
        out["ja"] = (sc["Kana"] + sc.get("Han", 0)) / letters
    elif sc.get("Han", 0):
        out["zh"] = sc["Han"] / letters
    if sc.get("CYRILLIC", 0):
        uk = any(ch in text for ch in "іїєґІЇЄҐ")
        # Bulgarian writes ъ as a vowel and has no ы / э: ъ without either marks it
        bg = not uk and any(ch in text for ch in "ъЪ") and not any(ch in text for ch in "ыЫэЭ")
        out["uk" if uk else ("bg" if bg else "ru")] = sc["CYRILLIC"] / letters
    if sc.get("ARABIC", 0):
        fa = any(ch in text for ch in "پچژگ\u06a9\u06cc")      # + keheh, farsi yeh
        out["fa" if fa else "ar"] = sc["ARABIC"] / letters
    for s, lang in _SCRIPT_LANG.items():
        if sc.get(s, 0):
            out[lang] = sc[s] / letters
    if latin:
        toks = TU.tokenize(text, stopwords=frozenset())
        hits = {lang: sum(1 for t in toks if t in words) for lang, words in PROFILES.items()}
        top = max(hits.values()) if hits else 0
        distinct = max((len(set(toks) & words) for words in PROFILES.values()), default=0)
        if distinct < 2 and len(out) and latin < letters:
            # Latin tokens with fewer than two distinct function words next to another script -- markup, names,
            # URLs: they identify nothing, so the other scripts' shares are taken among the rest of the letters
            rest = letters - latin
            return dict(sorted(((k, min(1.0, v * letters / rest)) for k, v in out.items()), key=lambda kv: -kv[1]))
        if top:
            # posterior of a naive token model: each profile hit multiplies a language's odds by _ODDS
            share = latin / letters
            w = {lang: _ODDS ** (h - top) for lang, h in hits.items() if h}
            z = sum(w.values())
            for lang, v in w.items():
                out[lang] = out.get(lang, 0.0) + share * v / z
    return dict(sorted(out.items(), key=lambda kv: -kv[1]))


def best_language(text: Optional[str], threshold: float = 0.99, default: str = UNKNOWN) -> str:
    """The top detected language when its confidence exceeds ``threshold``, else ``default``
    (``TextTokenizer.tokenize`` with autoDetectLanguage, ``TextTokenizer.scala:168-176``)."""
    langs = detect_languages(text)
    if langs:
        lang, conf = next(iter(langs.items()))
        if conf > threshold:
            return lang
    return default


# the reference's Language enum names (utils/.../text/Language.scala) -> the codes used here
LANGUAGE_NAMES = {"English": "en", "French": "fr", "German": "de", "Spanish": "es", "Italian": "it", "Portuguese": "pt",
                  "Brazilian": "pt", "Dutch": "nl", "Swedish": "sv", "Danish": "da", "Norwegian": "no", "Polish": "pl",
                  "Catalan": "ca", "Finnish": "fi", "Turkish": "tr", "Romanian": "ro", "Russian": "ru",
                  "Hungarian": "hu", "Japanese": "ja", "Korean": "ko", "SimplifiedChinese": "zh-cn",
                  "TraditionalChinese": "zh-tw", "Chinese": "zh", "Arabic": "ar",
                  "Hindi": "hi", "Bulgarian": "bg", "Czech": "cs",
                  "Persian": "fa", "Indonesian": "id", "Latvian": "lv", "Greek": "el", "Lithuanian": "lt",
                  "Galician": "gl", "Basque": "eu", "Irish": "ga", "Bengali": "bn", "Sorani": "ckb", "Thai": "th"}
LANGUAGE_NAMES["Brazilian"] = "pt-br"
# Lucene CJKAnalyzer languages (LuceneTextAnalyzer.scala: Korean, SimplifiedChinese, TraditionalChinese)
CJK_BIGRAM = frozenset({"zh", "zh-cn", "zh-tw", "ko"})


def _pre_stop_normalizers():
    from .stemmers import hindi_normalize, persian_normalize
    from .stemmers_more import PRE_STOP_MORE
    return {"hi": hindi_normalize, "fa": persian_normalize, **PRE_STOP_MORE}


_PRE_STOP_NORMALIZERS = _pre_stop_normalizers()


def analyze(text: str, language: str = UNKNOWN, to_lowercase: bool = True, min_token_length: int = 1) -> List[str]:
    """Per-language analysis: elision stripping (fr / it / ca), the language's stop words (English's for an
    unknown language, as the reference's default StandardAnalyzer), StandardAnalyzer word rules; Chinese and
    Korean through the CJKAnalyzer bigrams (:func:`utils.text.analyze_cjk_bigrams`). Japanese (Kuromoji
    morphology in the reference) keeps the StandardAnalyzer segmentation: parity unpinned."""
    language = LANGUAGE_NAMES.get(language, language)
    if language in CJK_BIGRAM:
        s = text.lower() if to_lowercase else text
        return [t for t in TU.analyze_cjk_bigrams(s, TU.ENGLISH_STOPWORDS) if len(t) >= min_token_length]
    lang = language if language in STOPWORDS else "en"
    if lang == "fa":              # PersianCharFilter: ZWNJ separates words
        text = text.replace("\u200c", " ")
    if lang == "tr":
        # StandardTokenizer keeps a word joined by ' or \u2019 whole, ApostropheFilter then drops the apostrophe
        # and what follows it (Türkiye'nin -> türkiye); TurkishLowerCaseFilter maps I -> ı and İ -> i
        text = text.replace("\u2019", "'")
        if to_lowercase:
            from .snowball import turkish_lower
            text = turkish_lower(text)
    if lang == "ga" and to_lowercase:
        # IrishLowerCaseFilter: an initial n / t before an upper-case vowel is a prefix (nAthair -> n-athair)
        import re
        text = re.sub(r"\b([nt])([AEIOU\u00c1\u00c9\u00cd\u00d3\u00da])", r"\1-\2", text)
    toks = TU.tokenize(text, to_lowercase, 1, stopwords=frozenset())
    if lang == "tr":
        toks = [t.partition("'")[0] for t in toks]
    el = _ELISIONS.get(lang)
    if el:
        out = []
        for t in toks:
            q = t.replace("\u2019", "'")        # ElisionFilter takes both apostrophes
            if "'" in q:
                head, _, tail = q.partition("'")
                if head.lower() in el and tail:
                    t = tail
            out.append(t)
        toks = out
    sw = STOPWORDS[lang]
    if language == "en":
        # EnglishAnalyzer: possessive removal, stop words, Porter stemming (the default, unknown-language
        # StandardAnalyzer does not stem)
        from .stemmer import english_possessive, porter_stem
        toks = [english_possessive(t) for t in toks]
        return [porter_stem(t) for t in toks if t not in sw and len(t) >= min_token_length]
    from .stemmers import STEMMERS
    stem = STEMMERS.get(language)
    if language in ("ar", "hi", "fa", "bn", "ckb"):  # DecimalDigitFilter: any Unicode decimal digit -> its ASCII digit
        toks = ["".join(str(unicodedata.digit(c)) if c.isdecimal() and not c.isascii() else c for c in t)
                for t in toks]
    # analyzers whose normalisation filters run before their stop filter (HindiAnalyzer, PersianAnalyzer)
    pre = _PRE_STOP_NORMALIZERS.get(language)
    if pre is not None:
        toks = [pre(t) for t in toks]
    kept = [t for t in toks if t not in sw]
    if stem is not None:          # the language's Lucene analyzer stems after its stop filter
        kept = [stem(t) for t in kept]
    return [t for t in kept if len(t) >= min_token_length]
